// The proof object across the boundary: the wire format
// and a field-by-field view that maps 1:1 onto p3_uni_stark::Proof<SC>
// ([EXT p3-uni-stark proof.rs], produced at bin/src/main.rs:80-86 and
// consumed by p3_uni_stark::verify at bin/src/main.rs:88-96):
//   Proof { commitments: { trace, quotient_chunks },
//           opened_values: { trace_local, trace_next, quotient_chunks },
//           opening_proof: FriProof { commit_phase_commits, query_proofs,
//                                     final_poly, pow_witness },
//           degree_bits }
// lsp_proof_get_view hands out flat, query-major arrays of Montgomery-form
// elements (the lsp_fr convention); lsp_proof_from_view and
// lsp_proof_deserialize rebuild a proof handle from them (e.g. a Proof<SC>
// produced elsewhere, for lsp_verify).  Everything here is host code and
// treats its input bytes as untrusted (tests/test_proof_view.py fuzzes it,
// tools/sanitize builds it under ASan/UBSan).
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "prove_internal.hpp"

namespace lsp {

// little-endian words and canonical field elements, written in one pass into a
// buffer sized up front
namespace {
struct Writer {
    uint8_t* p;
    void u32(uint32_t x) {
        for (int i = 0; i < 4; ++i) *p++ = (uint8_t)(x >> (8 * i));
    }
    void fr(const Fr& x) {
        // Montgomery form -> integer: one Montgomery reduction (a product by 1
        // without the product rows) on the 4 x 64-bit host arithmetic
        const Fr c = hp64::to_canonical(hp64::redc(hp64::from(x)));
        std::memcpy(p, c.v, 32);  // 32-bit words little-endian (x86-64 host)
        p += 32;
    }
    void frs(const std::vector<Fr>& v) {
        for (auto& x : v) fr(x);
    }
};

// bounds-checked reader: every overrun or non-canonical element sets `bad`
struct Reader {
    const uint8_t* b;
    size_t n, off = 0;
    bool bad = false;
    uint32_t u32() {
        if (bad || n - off < 4) {
            bad = true;
            return 0;
        }
        uint32_t x = 0;
        for (int i = 0; i < 4; ++i) x |= (uint32_t)b[off + i] << (8 * i);
        off += 4;
        return x;
    }
    Fr fr() {
        Fr c = fr_zero();
        if (bad || n - off < 32) {
            bad = true;
            return c;
        }
        for (int i = 0; i < 8; ++i) {
            uint32_t x = 0;
            for (int k = 0; k < 4; ++k) x |= (uint32_t)b[off + 4 * i + k] << (8 * k);
            c.v[i] = x;
        }
        off += 32;
        if (!fr_words_lt_mod(c)) {
            bad = true;
            return fr_zero();
        }
        return fr_from_canonical(c);
    }
    // n elements, refusing counts the remaining bytes cannot hold (no huge allocations)
    void frs(std::vector<Fr>& v, size_t cnt) {
        if (bad || cnt > (n - off) / 32) {
            bad = true;
            return;
        }
        v.resize(cnt);
        for (auto& x : v) x = fr();
    }
};
}  // namespace

namespace {
struct Recycler {
    std::mutex mu;
    std::vector<std::vector<uint8_t>> wires;
    std::vector<std::vector<lsp_query>> queries;
    static constexpr size_t KEEP = 4;  // proofs' worth held at most
};
Recycler& recycler() {
    static Recycler* r = new Recycler();  // never destroyed: frees may run during exit
    return *r;
}
}  // namespace

// LSP_RECYCLE=0: plain frees and fresh allocations (same-box A/B; read per call)
static bool recycle_on() {
    const char* e = std::getenv("LSP_RECYCLE");
    return !(e && *e == '0');
}

void proof_release(lsp_proof* p) {
    if (!p) return;
    if (!recycle_on()) {
        delete p;
        return;
    }
    Recycler& r = recycler();
    {
        std::lock_guard<std::mutex> g(r.mu);
        if (r.wires.size() < Recycler::KEEP && p->wire.capacity() > 0) r.wires.push_back(std::move(p->wire));
        if (r.queries.size() < Recycler::KEEP && p->queries.capacity() > 0) r.queries.push_back(std::move(p->queries));
    }
    delete p;
}

std::vector<uint8_t> recycled_wire() {
    if (!recycle_on()) return {};
    Recycler& r = recycler();
    std::lock_guard<std::mutex> g(r.mu);
    if (r.wires.empty()) return {};
    std::vector<uint8_t> v = std::move(r.wires.back());
    r.wires.pop_back();
    return v;
}

std::vector<lsp_query> recycled_queries() {
    if (!recycle_on()) return {};
    Recycler& r = recycler();
    std::lock_guard<std::mutex> g(r.mu);
    if (r.queries.empty()) return {};
    std::vector<lsp_query> v = std::move(r.queries.back());
    r.queries.pop_back();
    return v;
}

std::vector<uint8_t> serialize(const lsp_proof& p, HostPool* pool, std::vector<uint8_t>* reuse) {
    size_t nfr = 3 + p.tl.size() + p.tn.size() + p.qc.size() + p.roots.size() + p.final_poly.size(), nu32 = 6;
    // byte offset of every query's record (queries are written independently)
    std::vector<size_t> qoff(p.queries.size() + 1);
    size_t qbytes = 0;
    for (size_t i = 0; i < p.queries.size(); ++i) {
        const auto& q = p.queries[i];
        size_t f = q.trow.size() + q.tpath.size() + q.qrow.size() + q.qpath.size() + q.sib.size(), u = 2 + q.sib.size();
        for (auto& fp : q.fpath) f += fp.size();
        qoff[i] = qbytes;
        qbytes += 32 * f + 4 * u;
    }
    const size_t head = 8 + 4 * nu32 + 32 * nfr;  // header + the fields before the queries
    std::vector<uint8_t> b;
    if (reuse) b.swap(*reuse);
    // every byte is written below, so a recycled buffer needs no clearing
    // (resize value-initialises only what it adds)
    b.resize(head + qbytes);
    std::memcpy(b.data(), "LSPPRF02", 8);
    Writer w{b.data() + 8};
    w.u32(p.log_h);
    w.u32(p.log_q);
    w.u32(p.w);
    w.u32((uint32_t)p.queries.size());
    w.u32((uint32_t)p.roots.size());
    w.u32((uint32_t)p.final_poly.size());
    w.fr(p.troot);
    w.fr(p.qroot);
    w.frs(p.tl);
    w.frs(p.tn);
    w.frs(p.qc);
    w.frs(p.roots);
    w.frs(p.final_poly);
    w.fr(p.pow_w);
    if (w.p != b.data() + head) throw LspError(LSP_E_STATE, "proof serialization size mismatch");
    auto write_query = [&](size_t i) {
        const auto& q = p.queries[i];
        Writer wq{b.data() + head + qoff[i]};
        wq.frs(q.trow);
        wq.u32((uint32_t)q.tpath.size());
        wq.frs(q.tpath);
        wq.frs(q.qrow);
        wq.u32((uint32_t)q.qpath.size());
        wq.frs(q.qpath);
        for (size_t r = 0; r < q.sib.size(); ++r) {
            wq.fr(q.sib[r]);
            wq.u32((uint32_t)q.fpath[r].size());
            wq.frs(q.fpath[r]);
        }
    };
    if (pool && p.queries.size() > 1)
        pool->parallel_for(p.queries.size(), write_query);
    else
        for (size_t i = 0; i < p.queries.size(); ++i) write_query(i);
    return b;
}

// Untrusted bytes: every count is range-checked before anything is sized by
// it, and the buffer must be consumed exactly.
lsp_proof* deserialize(const uint8_t* buf, size_t len) {
    if (!buf || len < 8 + 24 || std::memcmp(buf, "LSPPRF02", 8) != 0)
        throw LspError(LSP_E_ARG, "not an LSPPRF02 proof");
    Reader r{buf, len};
    r.off = 8;
    auto p = std::make_unique<lsp_proof>();
    p->log_h = r.u32();
    p->log_q = r.u32();
    p->w = r.u32();
    const uint32_t nq = r.u32(), nr = r.u32(), nf = r.u32();
    if (r.bad || p->log_h > 40 || p->log_q > 20 || p->w == 0 || p->w > (1u << 20) || nr > 64 || nq > (1u << 20) ||
        nf == 0 || nf > (1u << 20) || (nf & (nf - 1)) != 0)
        throw LspError(LSP_E_ARG, "proof header out of range");
    const size_t q = (size_t)1 << p->log_q;
    p->troot = r.fr();
    p->qroot = r.fr();
    r.frs(p->tl, p->w);
    r.frs(p->tn, p->w);
    r.frs(p->qc, q);
    r.frs(p->roots, nr);
    r.frs(p->final_poly, nf);
    p->pow_w = r.fr();
    if (r.bad || nq > (len - r.off) / (32 * (p->w + q))) throw LspError(LSP_E_ARG, "malformed proof bytes");
    p->queries.resize(nq);
    for (auto& qq : p->queries) {
        r.frs(qq.trow, p->w);
        r.frs(qq.tpath, r.u32());
        r.frs(qq.qrow, q);
        r.frs(qq.qpath, r.u32());
        qq.sib.resize(nr);
        qq.fpath.resize(nr);
        for (uint32_t k = 0; k < nr && !r.bad; ++k) {
            qq.sib[k] = r.fr();
            r.frs(qq.fpath[k], r.u32());
        }
        if (r.bad) break;
    }
    if (r.bad || r.off != len) throw LspError(LSP_E_ARG, "malformed proof bytes");
    return p.release();
}

namespace {
// the flat arrays behind lsp_proof_view, built on first use and kept with the proof
struct Flat {
    std::vector<Fr> single;  // trace_commit, quotient_commit, pow_witness
    std::vector<Fr> trows, tpaths, qrows, qpaths, sibs, fpaths;
    std::vector<uint32_t> fri_path_lens;
    uint32_t input_path_len = 0;
};
}  // namespace

void proof_view(const lsp_proof& p, lsp_proof_view* v) {
    // built once, under the proof's cache mutex; never replaced afterwards, so
    // pointers handed out stay valid until lsp_proof_free
    std::lock_guard<std::mutex> g(p.cache_mu);
    if (!p.view_cache) {
        auto f = std::make_shared<Flat>();
        const size_t nq = p.queries.size(), nr = p.roots.size();
        f->single = {p.troot, p.qroot, p.pow_w};
        f->input_path_len = nq ? (uint32_t)p.queries[0].tpath.size() : 0;
        f->fri_path_lens.assign(nr, 0);
        if (nq && p.queries[0].fpath.size() != nr) throw LspError(LSP_E_STATE, "proof queries are not uniform");
        for (size_t k = 0; k < nr && nq; ++k) f->fri_path_lens[k] = (uint32_t)p.queries[0].fpath[k].size();
        for (auto& q : p.queries) {
            // the view holds one path length per tree (true of every proof
            // this library makes: all matrices of a tree have one height)
            if (q.tpath.size() != f->input_path_len || q.qpath.size() != f->input_path_len || q.sib.size() != nr ||
                q.fpath.size() != nr || q.trow.size() != p.w || q.qrow.size() != p.qc.size())
                throw LspError(LSP_E_STATE, "proof queries are not uniform");
            for (size_t k = 0; k < nr; ++k)
                if (q.fpath[k].size() != f->fri_path_lens[k]) throw LspError(LSP_E_STATE, "FRI paths differ in length");
            f->trows.insert(f->trows.end(), q.trow.begin(), q.trow.end());
            f->tpaths.insert(f->tpaths.end(), q.tpath.begin(), q.tpath.end());
            f->qrows.insert(f->qrows.end(), q.qrow.begin(), q.qrow.end());
            f->qpaths.insert(f->qpaths.end(), q.qpath.begin(), q.qpath.end());
            f->sibs.insert(f->sibs.end(), q.sib.begin(), q.sib.end());
            for (auto& fp : q.fpath) f->fpaths.insert(f->fpaths.end(), fp.begin(), fp.end());
        }
        p.view_cache = f;
    }
    const Flat& f = *std::static_pointer_cast<Flat>(p.view_cache);
    auto fr = [](const std::vector<Fr>& x) { return reinterpret_cast<const lsp_fr*>(x.data()); };
    auto fr1 = [](const Fr& x) { return reinterpret_cast<const lsp_fr*>(&x); };
    std::memset(v, 0, sizeof *v);
    v->degree_bits = p.log_h;
    v->log_quotient_chunks = p.log_q;
    v->width = p.w;
    v->num_queries = (uint32_t)p.queries.size();
    v->num_fri_rounds = (uint32_t)p.roots.size();
    v->final_poly_len = (uint32_t)p.final_poly.size();
    v->input_path_len = f.input_path_len;
    v->fri_path_lens = f.fri_path_lens.data();
    v->trace_commit = fr1(f.single[0]);
    v->quotient_commit = fr1(f.single[1]);
    v->pow_witness = fr1(f.single[2]);
    v->trace_local = fr(p.tl);
    v->trace_next = fr(p.tn);
    v->quotient_chunks = fr(p.qc);
    v->fri_commits = fr(p.roots);
    v->final_poly = fr(p.final_poly);
    v->trace_rows = fr(f.trows);
    v->trace_paths = fr(f.tpaths);
    v->quotient_rows = fr(f.qrows);
    v->quotient_paths = fr(f.qpaths);
    v->fri_siblings = fr(f.sibs);
    v->fri_paths = fr(f.fpaths);
}

lsp_proof* proof_from_view(const lsp_proof_view& v) {
    // final_poly_len: a power of two (1 << log_final_poly_len) <= 2^20, the
    // lengths the wire format's reader accepts, so every view that builds a
    // handle serializes to bytes lsp_proof_deserialize reads back
    if (v.width == 0 || v.width > (1u << 20) || v.log_quotient_chunks > 20 || v.degree_bits > 40 ||
        v.num_fri_rounds > 64 || v.input_path_len > 64 || v.final_poly_len == 0 || v.final_poly_len > (1u << 20) ||
        (v.final_poly_len & (v.final_poly_len - 1)) != 0)
        throw LspError(LSP_E_ARG, "proof view out of range");
    const size_t w = v.width, q = (size_t)1 << v.log_quotient_chunks, nr = v.num_fri_rounds, pl = v.input_path_len;
    LSP_REQUIRE(v.trace_commit && v.quotient_commit && v.pow_witness && v.trace_local && v.trace_next &&
                    v.quotient_chunks && (nr == 0 || (v.fri_commits && v.fri_path_lens)) && v.final_poly,
                LSP_E_ARG, "null proof view field");
    LSP_REQUIRE(v.num_queries == 0 || (v.trace_rows && v.quotient_rows && v.fri_siblings &&
                                       (pl == 0 || (v.trace_paths && v.quotient_paths))),
                LSP_E_ARG, "null proof view query field");
    size_t fsum = 0;
    for (size_t k = 0; k < nr; ++k) {
        LSP_REQUIRE(v.fri_path_lens[k] <= 64, LSP_E_ARG, "FRI path too long");
        fsum += v.fri_path_lens[k];
    }
    LSP_REQUIRE(fsum == 0 || v.num_queries == 0 || v.fri_paths, LSP_E_ARG, "null FRI paths");
    auto rd = [](const lsp_fr* x, size_t n) {
        const Fr* f = reinterpret_cast<const Fr*>(x);
        for (size_t i = 0; i < n; ++i)
            LSP_REQUIRE(fr_words_lt_mod(f[i]), LSP_E_ARG, "proof element not reduced below the modulus");
        return std::vector<Fr>(f, f + n);
    };
    auto p = std::make_unique<lsp_proof>();
    p->log_h = v.degree_bits;
    p->log_q = v.log_quotient_chunks;
    p->w = v.width;
    p->troot = rd(v.trace_commit, 1)[0];
    p->qroot = rd(v.quotient_commit, 1)[0];
    p->pow_w = rd(v.pow_witness, 1)[0];
    p->tl = rd(v.trace_local, w);
    p->tn = rd(v.trace_next, w);
    p->qc = rd(v.quotient_chunks, q);
    p->roots = nr ? rd(v.fri_commits, nr) : std::vector<Fr>();
    p->final_poly = rd(v.final_poly, v.final_poly_len);
    p->queries.resize(v.num_queries);
    for (size_t i = 0; i < v.num_queries; ++i) {
        auto& qq = p->queries[i];
        qq.trow = rd(v.trace_rows + i * w, w);
        qq.tpath = pl ? rd(v.trace_paths + i * pl, pl) : std::vector<Fr>();
        qq.qrow = rd(v.quotient_rows + i * q, q);
        qq.qpath = pl ? rd(v.quotient_paths + i * pl, pl) : std::vector<Fr>();
        qq.sib = nr ? rd(v.fri_siblings + i * nr, nr) : std::vector<Fr>();
        qq.fpath.resize(nr);
        size_t o = i * fsum;
        for (size_t k = 0; k < nr; ++k) {
            qq.fpath[k] = v.fri_path_lens[k] ? rd(v.fri_paths + o, v.fri_path_lens[k]) : std::vector<Fr>();
            o += v.fri_path_lens[k];
        }
    }
    return p.release();
}

}  // namespace lsp
