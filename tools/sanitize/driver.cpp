// Host-side fuzz driver for the untrusted-input parsers of liblsp_hip.so,
// built and run under ASan + UBSan by tools/sanitize/run.sh (host code only;
// no GPU is touched: a verifier-only context, LSP_HOST_ONLY).
//
//   driver <seed> <iterations> <proof.bin> <trace.cbor>...
//
// For each input: the unmodified bytes, every truncation at a stride, and
// <iterations> random mutations (byte flips, spliced length fields, appended
// garbage) go through
//   lsp_raw_trace_parse (+ lsp_raw_trace_shape / _columns)  -- cbor.cpp
//   lsp_proof_deserialize (+ get_view / from_view / serialize round trip) and
//   lsp_verify on a host-only context                        -- proof.cpp, verify.cpp
//   lsp_fr_from_be_bytes_mod_order on random lengths          -- host field code
// Any out-of-bounds access, leak-free UB or overflow aborts under the
// sanitizers; logic failures (a parsed proof that does not re-serialize to
// its input, an accepted corrupted proof) exit 1.
#include <lsp.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <vector>

static std::vector<uint8_t> slurp(const char* path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        std::fprintf(stderr, "cannot read %s\n", path);
        std::exit(2);
    }
    return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
}

static std::vector<std::vector<uint8_t>> variants(const std::vector<uint8_t>& b, std::mt19937_64& rng, int iters) {
    std::vector<std::vector<uint8_t>> out;
    out.push_back(b);
    const size_t stride = b.size() > 64 ? b.size() / 64 : 1;
    for (size_t k = 0; k < b.size(); k += stride) out.emplace_back(b.begin(), b.begin() + k);
    for (int it = 0; it < iters; ++it) {
        std::vector<uint8_t> m = b;
        const int kind = (int)(rng() % 4);
        if (m.empty()) m.push_back(0);
        if (kind == 0) {  // 1-4 random bytes
            for (int j = 1 + (int)(rng() % 4); j > 0; --j) m[rng() % m.size()] = (uint8_t)rng();
        } else if (kind == 1) {  // a 32-bit little-endian field set to an extreme
            const uint32_t vals[] = {0u, 1u, 0x7fffffffu, 0xffffffffu, 1u << 20, 1u << 31};
            const size_t off = rng() % m.size();
            const uint32_t v = vals[rng() % 6];
            for (int j = 0; j < 4 && off + j < m.size(); ++j) m[off + j] = (uint8_t)(v >> (8 * j));
        } else if (kind == 2) {  // a CBOR-style head byte with a huge length argument
            const size_t off = rng() % m.size();
            m[off] = (uint8_t)((rng() % 8) << 5 | (24 + rng() % 4));
        } else {  // garbage appended or a chunk deleted
            if (rng() % 2)
                for (int j = (int)(rng() % 40); j > 0; --j) m.push_back((uint8_t)rng());
            else if (m.size() > 2) {
                const size_t a = rng() % m.size(), len = 1 + rng() % (m.size() - a);
                m.erase(m.begin() + a, m.begin() + a + len);
            }
        }
        out.push_back(std::move(m));
    }
    return out;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s seed iterations proof.bin [trace.cbor...]\n", argv[0]);
        return 2;
    }
    std::mt19937_64 rng(std::strtoull(argv[1], nullptr, 10));
    const int iters = std::atoi(argv[2]);
    size_t runs = 0, parsed_ok = 0;

    // ---- proofs: deserialize, view round trip, verify
    std::vector<lsp_fr> rc(3 * 8 + 22);
    lsp_fr alpha, delta;
    if (lsp_seeded_setup(0x4C494E4541ull, 8, 22, &alpha, &delta, rc.data()) != LSP_OK) return 3;
    lsp_params prm{};
    prm.struct_size = sizeof prm;
    prm.sbox_degree = 11;
    prm.rounds_f = 8;
    prm.rounds_p = 22;
    prm.round_constants = rc.data();
    prm.log_blowup = 3;
    prm.num_queries = 33;
    prm.public_degree = 1;
    const char* nq = std::getenv("LSP_SAN_QUERIES");
    if (nq) prm.num_queries = (uint32_t)std::atoi(nq);
    lsp_ctx* ctx = nullptr;
    if (lsp_ctx_create(LSP_HOST_ONLY, &prm, &ctx) != LSP_OK) return 3;
    const int ncols = std::getenv("LSP_SAN_NCOLS") ? std::atoi(std::getenv("LSP_SAN_NCOLS")) : 3;
    std::vector<int32_t> air = {1, 1, ncols, ncols};
    for (int i = 0; i < 2 * ncols; ++i) air.push_back(i);
    air.push_back(2 * ncols);
    air.push_back(2 * ncols + 1);
    const lsp_fr pub[2] = {alpha, delta};
    const std::vector<uint8_t> proof = slurp(argv[3]);
    for (const auto& v : variants(proof, rng, iters)) {
        ++runs;
        lsp_proof* p = nullptr;
        const int rc1 = lsp_proof_deserialize(v.data(), v.size(), &p);
        if (rc1 == LSP_OK) {
            ++parsed_ok;
            lsp_proof_view view;
            size_t n = 0;
            lsp_proof* q = nullptr;
            if (lsp_proof_get_view(p, &view) == LSP_OK && lsp_proof_from_view(&view, &q) == LSP_OK) {
                std::vector<uint8_t> back;
                lsp_proof_serialize(q, nullptr, 0, &n);
                back.resize(n);
                lsp_proof_serialize(q, back.data(), n, &n);
                if (back != v) {
                    std::fprintf(stderr, "view round trip changed a proof (%zu bytes)\n", v.size());
                    return 1;
                }
                lsp_proof_free(q);
            }
            lsp_proof_free(p);
        } else if (rc1 != LSP_E_ARG) {
            std::fprintf(stderr, "lsp_proof_deserialize returned %d\n", rc1);
            return 1;
        }
        const int rcv = lsp_verify(ctx, air.data(), air.size(), pub, 2, v.data(), v.size());
        if (rcv == LSP_OK && v != proof) {
            std::fprintf(stderr, "a corrupted proof was accepted\n");
            return 1;
        }
        if (rcv != LSP_OK && v == proof) {
            std::fprintf(stderr, "the genuine proof was rejected: %s\n", lsp_last_error(nullptr));
            return 1;
        }
    }

    // ---- CBOR traces
    for (int a = 4; a < argc; ++a) {
        const std::vector<uint8_t> t = slurp(argv[a]);
        for (const auto& v : variants(t, rng, iters)) {
            ++runs;
            lsp_raw_trace* rt = nullptr;
            const int r = lsp_raw_trace_parse(v.data(), v.size(), &rt);
            if (r == LSP_OK) {
                int kind;
                uint32_t na, nt, nbc;
                size_t mh, w, n = 0;
                lsp_raw_trace_shape(rt, &kind, &na, &nt, &nbc, &mh, &w);
                if (mh <= (1u << 16)) {
                    lsp_raw_trace_columns(rt, mh, nullptr, 0, &n);
                    std::vector<lsp_fr> cols(n);
                    lsp_raw_trace_columns(rt, mh, cols.data(), n, &n);
                }
                lsp_raw_trace_free(rt);
            } else if (r != LSP_E_ARG && r != LSP_E_SIZE) {
                std::fprintf(stderr, "lsp_raw_trace_parse returned %d\n", r);
                return 1;
            }
        }
    }

    // ---- big-endian words of every length
    for (int it = 0; it < 200; ++it) {
        std::vector<uint8_t> be(rng() % 80);
        for (auto& x : be) x = (uint8_t)rng();
        lsp_fr out;
        lsp_fr_from_be_bytes_mod_order(be.data(), be.size(), &out);
    }
    lsp_ctx_destroy(ctx);
    std::printf("sanitize ok: %zu inputs, %zu proofs parsed\n", runs, parsed_ok);
    return 0;
}
