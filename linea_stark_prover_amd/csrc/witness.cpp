// Host witness generation for synthetic traces -- the reference's `trace`
// crate semantics (RawPermutationTrace::get_trace, trace/src/permutation.rs:24-93;
// RawLookupTrace::get_trace, trace/src/lookup.rs:46-176; RawTrace::push_traces /
// get_trace, trace/src/lib.rs:62-106), used to build the wide-AIR workload
// (the stand-in for the missing zkevm.bin).
//
// Layout follows RawTrace: lookup traces first, then permutation traces
// (trace/src/lib.rs:81-89), each config shifted by the columns already pushed.
#include <algorithm>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "prove_internal.hpp"

namespace lsp {
namespace {
struct Rng {  // SplitMix64 (U4), same as the seeded setup
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    Fr fr() {
        for (;;) {
            Fr c;
            for (int k = 0; k < 4; ++k) {
                const uint64_t x = next();
                c.v[2 * k] = (uint32_t)x;
                c.v[2 * k + 1] = (uint32_t)(x >> 32);
            }
            c.v[7] &= (1u << 29) - 1;
            if (fr_words_lt_mod(c)) return fr_from_canonical(c);
        }
    }
    uint64_t below(uint64_t n) {
        const unsigned __int128 two64 = (unsigned __int128)1 << 64;
        const unsigned __int128 lim = two64 - (two64 % n);
        for (;;) {
            const uint64_t x = next();
            if ((unsigned __int128)x < lim) return x % n;
        }
    }
};

struct FrHash {
    size_t operator()(const Fr& x) const {
        uint64_t h = 0xcbf29ce484222325ull;
        for (int i = 0; i < 8; ++i) h = (h ^ x.v[i]) * 0x100000001b3ull;
        return (size_t)h;
    }
};
struct FrEq {
    bool operator()(const Fr& a, const Fr& b) const { return fr_eq(a, b); }
};

void batch_inv(std::vector<Fr>& v) {
    std::vector<Fr> pre(v.size());
    Fr acc = fr_one();
    for (size_t i = 0; i < v.size(); ++i) {
        pre[i] = acc;
        acc = fr_mul(acc, v[i]);
    }
    Fr inv = fr_inv(acc);
    for (size_t i = v.size(); i-- > 0;) {
        const Fr t = fr_mul(inv, pre[i]);
        inv = fr_mul(inv, v[i]);
        v[i] = t;
    }
}

Fr combo(const std::vector<std::vector<Fr>>& cols, size_t i, const Fr& alpha) {
    Fr acc = fr_zero();
    for (const auto& c : cols) acc = fr_add(fr_mul(acc, alpha), c[i]);
    return acc;
}
}  // namespace

// RawLookupTrace::get_trace: columns a.., b tables.., a_filter, b_filters..,
// a_inverses, b_inverses.., multiplicities.., prefix sum
static void lookup_columns(const std::vector<std::vector<Fr>>& a, const std::vector<std::vector<std::vector<Fr>>>& b,
                           const std::vector<Fr>& a_filter, const std::vector<std::vector<Fr>>& b_filter,
                           const Fr& alpha, const Fr& delta, std::vector<std::vector<Fr>>& out, size_t shift,
                           std::vector<int32_t>& desc) {
    const size_t n = a[0].size(), na = a.size(), nt = b.size(), nbc = b[0].size();
    const Fr zero = fr_zero();
    std::unordered_map<Fr, uint64_t, FrHash, FrEq> occ;
    std::vector<Fr> acomb(n);
    for (size_t i = 0; i < n; ++i) {
        acomb[i] = combo(a, i, alpha);
        if (!fr_eq(a_filter[i], zero)) occ[acomb[i]] += 1;
    }
    std::vector<Fr> a_inv(n);
    for (size_t i = 0; i < n; ++i) a_inv[i] = fr_add(acomb[i], delta);
    batch_inv(a_inv);
    std::vector<std::vector<Fr>> bcomb(nt, std::vector<Fr>(n)), b_inv(nt, std::vector<Fr>(n)),
        mult(nt, std::vector<Fr>(n, zero));
    for (size_t t = 0; t < nt; ++t) {
        for (size_t i = 0; i < n; ++i) {
            bcomb[t][i] = combo(b[t], i, alpha);
            b_inv[t][i] = fr_add(bcomb[t][i], delta);
        }
        batch_inv(b_inv[t]);
    }
    std::vector<Fr> psum(n);
    Fr s = zero;
    for (size_t i = 0; i < n; ++i) {
        if (!fr_eq(a_filter[i], zero)) s = fr_add(s, a_inv[i]);
        for (size_t t = 0; t < nt; ++t) {
            auto it = occ.find(bcomb[t][i]);
            if (it != occ.end() && !fr_eq(b_filter[t][i], zero)) {
                const Fr o = fr_from_u64(it->second);
                s = fr_sub(s, fr_mul(b_inv[t][i], o));
                mult[t][i] = o;
                occ.erase(it);
            }
        }
        psum[i] = s;
    }
    LSP_REQUIRE(fr_is_zero(psum[n - 1]), LSP_E_STATE,
                "failed to check constrain: check column should be 0 on the last row");
    // column ids (trace/src/lookup.rs:178-214), shifted
    const int32_t base = (int32_t)shift;
    desc.push_back(LSP_AIR_LOOKUP);
    desc.push_back((int32_t)na);
    for (size_t c = 0; c < na; ++c) desc.push_back(base + (int32_t)c);
    desc.push_back((int32_t)nt);
    desc.push_back((int32_t)nbc);
    for (size_t i = 0; i < nt * nbc; ++i) desc.push_back(base + (int32_t)(na + i));
    const int32_t a_filter_id = base + (int32_t)(na + nt * nbc);
    desc.push_back(a_filter_id);
    for (size_t t = 0; t < nt; ++t) desc.push_back(a_filter_id + 1 + (int32_t)t);
    const int32_t a_inv_id = a_filter_id + (int32_t)nt + 1;
    desc.push_back(a_inv_id);
    for (size_t t = 0; t < nt; ++t) desc.push_back(a_inv_id + 1 + (int32_t)t);
    for (size_t t = 0; t < nt; ++t) desc.push_back(a_inv_id + 1 + (int32_t)nt + (int32_t)t);
    desc.push_back(a_inv_id + 1 + 2 * (int32_t)nt);
    for (auto& c : a) out.push_back(c);
    for (auto& tab : b)
        for (auto& c : tab) out.push_back(c);
    out.push_back(a_filter);
    for (auto& f : b_filter) out.push_back(f);
    out.push_back(a_inv);
    for (auto& c : b_inv) out.push_back(c);
    for (auto& c : mult) out.push_back(c);
    out.push_back(psum);
}

// RawPermutationTrace::get_trace: columns a.., b.., b_inverse, check
static void permutation_columns(const std::vector<std::vector<Fr>>& a, const std::vector<std::vector<Fr>>& b,
                                const Fr& alpha, const Fr& delta, std::vector<std::vector<Fr>>& out, size_t shift,
                                std::vector<int32_t>& desc) {
    const size_t n = a[0].size(), w = a.size();
    std::vector<Fr> binv(n), chk(n);
    for (size_t i = 0; i < n; ++i) binv[i] = fr_add(combo(b, i, alpha), delta);
    batch_inv(binv);
    Fr prev = fr_one();
    for (size_t i = 0; i < n; ++i) {
        prev = fr_mul(fr_mul(prev, fr_add(combo(a, i, alpha), delta)), binv[i]);
        chk[i] = prev;
    }
    LSP_REQUIRE(fr_eq(prev, fr_one()), LSP_E_STATE,
                "failed to check constrain: check column should be 1 on the last row");
    const int32_t base = (int32_t)shift;
    desc.push_back(LSP_AIR_PERMUTATION);
    desc.push_back((int32_t)w);
    desc.push_back((int32_t)w);
    for (size_t c = 0; c < 2 * w; ++c) desc.push_back(base + (int32_t)c);
    desc.push_back(base + 2 * (int32_t)w);
    desc.push_back(base + 2 * (int32_t)w + 1);
    for (auto& c : a) out.push_back(c);
    for (auto& c : b) out.push_back(c);
    out.push_back(binv);
    out.push_back(chk);
}

// The wide synthetic trace: nlookup LogUp lookups (A of
// `na` columns drawn from ntab tables of na columns each) followed by nperm
// permutation groups of pcols+pcols columns.  Deterministic in `seed`.
void gen_wide_trace(uint64_t seed, uint32_t log_n, uint32_t nlookup, uint32_t na, uint32_t ntab, uint32_t nperm,
                    uint32_t pcols, const Fr& alpha, const Fr& delta, std::vector<Fr>& rows, size_t& width,
                    std::vector<int32_t>& desc) {
    const size_t n = (size_t)1 << log_n;
    Rng g{seed ^ 0x57494445ull};  // "WIDE"
    std::vector<std::vector<Fr>> cols;
    desc.assign(1, (int32_t)(nlookup + nperm));
    for (uint32_t l = 0; l < nlookup; ++l) {
        std::vector<std::vector<std::vector<Fr>>> b(ntab, std::vector<std::vector<Fr>>(na, std::vector<Fr>(n)));
        for (auto& tab : b)
            for (auto& c : tab)
                for (auto& x : c) x = g.fr();
        std::vector<std::vector<Fr>> a(na, std::vector<Fr>(n));
        for (size_t i = 0; i < n; ++i) {
            const size_t t = (size_t)g.below(ntab), j = (size_t)g.below(n);
            for (uint32_t c = 0; c < na; ++c) a[c][i] = b[t][c][j];
        }
        std::vector<Fr> af(n, fr_one());
        std::vector<std::vector<Fr>> bf(ntab, std::vector<Fr>(n, fr_one()));
        lookup_columns(a, b, af, bf, alpha, delta, cols, cols.size(), desc);
    }
    for (uint32_t p = 0; p < nperm; ++p) {
        std::vector<std::vector<Fr>> a(pcols, std::vector<Fr>(n)), b(pcols, std::vector<Fr>(n));
        for (auto& c : a)
            for (auto& x : c) x = g.fr();
        std::vector<size_t> perm(n);
        for (size_t i = 0; i < n; ++i) perm[i] = i;
        for (size_t i = n - 1; i > 0; --i) std::swap(perm[i], perm[(size_t)g.below(i + 1)]);
        for (uint32_t c = 0; c < pcols; ++c)
            for (size_t i = 0; i < n; ++i) b[c][i] = a[c][perm[i]];
        permutation_columns(a, b, alpha, delta, cols, cols.size(), desc);
    }
    // RawTrace::get_trace: row-major, columns in push order (trace/src/lib.rs:94-106)
    width = cols.size();
    rows.resize(n * width);
    for (size_t i = 0; i < n; ++i)
        for (size_t c = 0; c < width; ++c) rows[i * width + c] = cols[c][i];
}

}  // namespace lsp

extern "C" int lsp_gen_wide_trace(uint64_t seed, uint32_t log_n, uint32_t nlookup, uint32_t na, uint32_t ntab,
                                  uint32_t nperm, uint32_t pcols, const lsp_fr* alpha, const lsp_fr* delta,
                                  lsp_fr* rows_out, size_t rows_cap, int32_t* air_out, size_t air_cap,
                                  size_t* width_out, size_t* air_len_out) {
    try {
        LSP_REQUIRE(alpha && delta && width_out && air_len_out && log_n >= 1 && log_n <= 26 &&
                        (nlookup == 0 || (na >= 1 && ntab >= 1)) && (nperm == 0 || pcols >= 1) &&
                        nlookup + nperm >= 1,
                    LSP_E_ARG, "bad wide-trace arguments");
        // sizes first (cheap): width = nlookup*(na + ntab*(na+3) + 3) + nperm*(2*pcols + 2)
        const size_t w = (size_t)nlookup * (na + (size_t)ntab * (na + 3) + 3) + (size_t)nperm * (2 * pcols + 2);
        const size_t dl = 1 + (size_t)nlookup * (5 + na + (size_t)ntab * na + 3 * ntab + 2) +
                          (size_t)nperm * (3 + 2 * pcols + 2);
        *width_out = w;
        *air_len_out = dl;
        if (!rows_out) return LSP_OK;
        LSP_REQUIRE(rows_cap >= ((size_t)1 << log_n) * w && air_out && air_cap >= dl, LSP_E_ARG,
                    "output buffers too small");
        std::vector<lsp::Fr> rows;
        std::vector<int32_t> desc;
        size_t width = 0;
        lsp::gen_wide_trace(seed, log_n, nlookup, na, ntab, nperm, pcols, lsp::to_fr(*alpha), lsp::to_fr(*delta),
                            rows, width, desc);
        LSP_REQUIRE(width == w && desc.size() == dl, LSP_E_STATE, "wide trace layout mismatch");
        std::memcpy(rows_out, rows.data(), rows.size() * sizeof(lsp::Fr));
        std::memcpy(air_out, desc.data(), desc.size() * sizeof(int32_t));
        return LSP_OK;
    } catch (const lsp::LspError& e) {
        return e.code;
    } catch (...) {
        return LSP_E_STATE;
    }
}

// ------------------------------------------------- device witness (F1)
namespace lsp {
// RawPermutationTrace::get_trace on the device: columns a.., b.., b_inverse,
// check (prefix product of (a_comb + delta) / (b_comb + delta), must end at 1)
void witness_permutation_device(lsp_ctx* ctx, const Fr* a, uint32_t na, const Fr* b, uint32_t nb, size_t n,
                                const Fr& alpha, const Fr& delta, Fr* out, size_t ostride) {
    hipStream_t st = ctx->stream;
    Fr* al = ctx->fbuf("wit_al", n);
    Fr* bl = ctx->fbuf("wit_bl", n);
    Fr* binv = ctx->fbuf("wit_binv", n);
    Fr* chk = ctx->fbuf("wit_chk", n);
    const size_t sb = witness_scratch_bytes(n, 0);
    void* scratch = ctx->buf("wit_scratch", sb);
    LSP_HIP(launch_perm_rows(a, na, b, nb, n, alpha, delta, out, ostride, al, bl, st));
    LSP_HIP(launch_batch_inverse(bl, binv, n, st, ctx->bi_scratch(n)));
    LSP_HIP(launch_mul_vec(al, binv, n, al, st));
    LSP_HIP(launch_fr_scan(al, chk, n, true, scratch, sb, st));
    LSP_HIP(launch_put_col(binv, n, out, ostride, na + nb, st));
    LSP_HIP(launch_put_col(chk, n, out, ostride, na + nb + 1, st));
    Fr last;
    LSP_HIP(hipMemcpyAsync(&last, chk + n - 1, sizeof(Fr), hipMemcpyDeviceToHost, st));
    LSP_HIP(hipStreamSynchronize(st));
    LSP_REQUIRE(fr_eq(last, fr_one()), LSP_E_STATE,
                "failed to check constrain: check column should be 1 on the last row");
}

// RawLookupTrace::get_trace on the device: columns a.., b tables.., a_filter,
// b_filters.., a_inverses, b_inverses.., multiplicities.., prefix sum (must end at 0)
void witness_lookup_device(lsp_ctx* ctx, const Fr* a, uint32_t na, const Fr* b, uint32_t nt, uint32_t nbc,
                           const Fr* afil, const Fr* bfil, size_t n, const Fr& alpha, const Fr& delta, Fr* out,
                           size_t ostride) {
    hipStream_t st = ctx->stream;
    const size_t m = n * (1 + (size_t)nt);
    Fr* comb = ctx->fbuf("wit_comb", m);
    Fr* den = ctx->fbuf("wit_den", m);
    Fr* inv = ctx->fbuf("wit_inv", m);
    uint32_t* occ = (uint32_t*)ctx->buf("wit_occ", std::max<size_t>(1, n * nt) * sizeof(uint32_t));
    Fr* term = ctx->fbuf("wit_term", n);
    Fr* psum = ctx->fbuf("wit_psum", n);
    const size_t sb = witness_scratch_bytes(n, nt);
    void* scratch = ctx->buf("wit_scratch", sb);
    LSP_HIP(launch_lookup_rows(a, na, b, nt, nbc, afil, bfil, n, alpha, delta, out, ostride, comb, den, st));
    LSP_HIP(launch_batch_inverse(den, inv, m, st, ctx->bi_scratch(m)));
    LSP_HIP(launch_lookup_occurrences(comb, n, nt, afil, bfil, occ, scratch, sb, st));
    const uint32_t col_ainv = na + nt * nbc + 1 + nt;
    LSP_HIP(launch_lookup_terms(inv, occ, afil, n, nt, out, ostride, col_ainv, term, st));
    LSP_HIP(launch_fr_scan(term, psum, n, false, scratch, sb, st));
    LSP_HIP(launch_put_col(psum, n, out, ostride, col_ainv + 1 + 2 * nt, st));
    Fr last;
    LSP_HIP(hipMemcpyAsync(&last, psum + n - 1, sizeof(Fr), hipMemcpyDeviceToHost, st));
    LSP_HIP(hipStreamSynchronize(st));
    LSP_REQUIRE(fr_is_zero(last), LSP_E_STATE, "failed to check constrain: check column should be 0 on the last row");
}
}  // namespace lsp
