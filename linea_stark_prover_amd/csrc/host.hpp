// Host-side internals of liblsp_hip.so: context, device buffer pool,
// transcript (HashChallenger), proof object.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <tuple>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/lsp.h"
#include "fr.hpp"
#include "kernels.hpp"
#include "poseidon2.hpp"
#include "poseidon2_host64.hpp"

namespace lsp {

struct LspError : std::runtime_error {
    int code;
    LspError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#ifdef LSP_DEBUG_BOUNDS
// the debug-bounds build checks the kernels' fault words after every HIP call
// (a device sync each), so a failed check names the launch that made it
// (capi.cpp; dbg_bounds.hpp)
void dbg_check_after(const char* what);  // (inside namespace lsp)
#define LSP_DBG_AFTER(x) ::lsp::dbg_check_after(x)
#else
#define LSP_DBG_AFTER(x) ((void)0)
#endif

#define LSP_HIP(x)                                                                                  \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess)                                                                       \
            throw ::lsp::LspError(LSP_E_HIP, std::string(#x) + " -> " + hipGetErrorString(e_)); \
        LSP_DBG_AFTER(#x);                                                                          \
    } while (0)

#define LSP_REQUIRE(cond, code, msg)                          \
    do {                                                      \
        if (!(cond)) throw ::lsp::LspError((code), (msg));    \
    } while (0)

inline Fr to_fr(const lsp_fr& x) {
    Fr r;
    for (int i = 0; i < 4; ++i) {
        r.v[2 * i] = (uint32_t)x.l[i];
        r.v[2 * i + 1] = (uint32_t)(x.l[i] >> 32);
    }
    return r;
}
inline lsp_fr from_fr(const Fr& x) {
    lsp_fr r;
    for (int i = 0; i < 4; ++i) r.l[i] = (uint64_t)x.v[2 * i] | ((uint64_t)x.v[2 * i + 1] << 32);
    return r;
}

// GENERATOR = 22 (U9) and two-adic generators
Fr host_generator();
Fr host_two_adic_generator(uint32_t bits);
// 1/a for the per-shape constants the prover inverts on its critical path
// (1/h, w^-1, 1/Z_H on the quotient cosets, ...): a process-wide cache, so a
// proof of a shape seen before spends no host time on Fermat inverses
Fr host_inv_cached(const Fr& a);
uint64_t host_bitrev(uint64_t x, uint32_t bits);
uint32_t log2_exact(size_t n);  // throws LSP_E_SIZE on non-power-of-two

// Poseidon2 on the host 8 at a time with AVX-512 IFMA (host_ifma.cpp); only
// when available() -- the CPU has avx512f + avx512ifma and LSP_HOST_IFMA != 0
namespace ifma {
struct alignas(64) Lane8 {  // one 52-bit limb of a value in 8 lanes (a __m512i)
    uint64_t w[8];
};
bool available();
void prepare(const std::vector<Fr>& rc, std::vector<Lane8>& rc_ifma);
// out[j] = compress(left[j * stride], right[j * stride]), j < n <= 8
void compress8(const Fr* left, const Fr* right, size_t stride, Fr* out, int n, const std::vector<Lane8>& rc,
               const P2Layout& L);
// the same for n <= 16, as two 8-lane states in lockstep
void compress16(const Fr* left, const Fr* right, size_t stride, Fr* out, int n, const std::vector<Lane8>& rc,
                const P2Layout& L);
// out[j] = hash_iter(rows[j * w .. j * w + w)), j < n <= 8
void hash8(const Fr* rows, size_t w, Fr* out, int n, const std::vector<Lane8>& rc, const P2Layout& L);
}  // namespace ifma

struct P2Host {
    P2Layout L;
    std::vector<Fr> rc;
    std::vector<ifma::Lane8> rc8;  // round constants for ifma::, 5 limbs each (empty: scalar only)
    // 4 x 64-bit limbs, lazily reduced (poseidon2_host64.hpp); canonical in and out
    void permute(Fr& s0, Fr& s1, Fr& s2) const { hp64::permute3_rt(s0, s1, s2, rc.data(), L); }
    Fr hash(const Fr* in, size_t n) const;
    Fr compress(const Fr& l, const Fr& r) const {
        Fr s0 = l, s1 = r, s2 = fr_zero();
        permute(s0, s1, s2);
        return s0;
    }
    // out[i] = compress(in[2i], in[2i+1]) for i in [i0, i1), 16 or 8 at a time when IFMA is there
    void compress_range(const Fr* in, Fr* out, size_t i0, size_t i1) const {
        if (rc8.empty()) {
            for (size_t i = i0; i < i1; ++i) out[i] = compress(in[2 * i], in[2 * i + 1]);
            return;
        }
        size_t i = i0;
        for (; i + 8 < i1; i += 16)  // two states in lockstep: ~10 % more per thread than 8 at a time
            ifma::compress16(in + 2 * i, in + 2 * i + 1, 2, out + i, (int)std::min<size_t>(16, i1 - i), rc8, L);
        if (i < i1) ifma::compress8(in + 2 * i, in + 2 * i + 1, 2, out + i, (int)(i1 - i), rc8, L);
    }
    // out[i] = hash(rows[i w ..]) for i in [i0, i1)
    void hash_range(const Fr* rows, size_t w, Fr* out, size_t i0, size_t i1) const {
        if (rc8.empty()) {
            for (size_t i = i0; i < i1; ++i) out[i] = hash(rows + i * w, w);
            return;
        }
        for (size_t i = i0; i < i1; i += 8)
            ifma::hash8(rows + i * w, w, out + i, (int)std::min<size_t>(8, i1 - i), rc8, L);
    }
};

// The transcript conventions of include/lsp.h's lsp_params (U7, U8, U12),
// each a named switch; the defaults are SURVEY 8(c)'s
struct TranscriptCfg {
    bool log_degree = true;      // U7: observe log2(h) first
    bool public_values = true;   // U7: observe the public values before alpha
    bool opened_values = false;  // U7: observe the opened values before alpha_fri
    bool mont_bits = false;      // U8: sample_bits from the Montgomery form
    bool final_poly = true;      // U12: observe the final polynomial
};

// HashChallenger<Val, Hash, 1> (bin/src/config.rs:23): input buffer,
// output buffer, hash_iter on flush with the output chained back as input.
struct Challenger {
    const P2Host* p2;
    std::vector<Fr> in, out;
    bool mont_bits = false;  // U8 (TranscriptCfg::mont_bits)
    explicit Challenger(const P2Host* p, bool mont = false) : p2(p), mont_bits(mont) {}
    void observe(const Fr& x) {
        out.clear();
        in.push_back(x);
    }
    Fr sample() {
        if (out.empty()) {
            Fr h = p2->hash(in.data(), in.size());
            in.assign(1, h);
            out.assign(1, h);
        }
        Fr r = out.back();
        out.pop_back();
        return r;
    }
    // U8: low bits of the canonical value (mont_bits: of the Montgomery form)
    uint64_t sample_bits(uint32_t bits) {
        const Fr s = sample();
        const Fr c = mont_bits ? s : fr_to_canonical(s);
        uint64_t lo = (uint64_t)c.v[0] | ((uint64_t)c.v[1] << 32);
        return bits >= 64 ? lo : (lo & ((1ull << bits) - 1));
    }
    bool check_witness(uint32_t bits, uint64_t w) {
        observe(fr_from_u64(w));
        return sample_bits(bits) == 0;
    }
    uint64_t grind(uint32_t bits) {
        for (uint64_t w = 0;; ++w) {
            Challenger probe = *this;
            if (probe.check_witness(bits, w)) {
                check_witness(bits, w);
                return w;
            }
        }
    }
};

struct AirCfg {
    int type;  // 1 perm, 2 lookup
    std::vector<int32_t> a, b;             // perm: a, b ; lookup: a, flattened b tables
    int32_t binv = 0, check = 0;           // perm
    int32_t ntab = 0, nbc = 0, a_filter = 0, a_inv = 0;
    std::vector<int32_t> b_filter, b_inv, occ;
};
struct Air {
    std::vector<AirCfg> cfgs;
    std::vector<int32_t> raw;
    uint32_t max_col = 0;
    static Air parse(const int32_t* d, size_t n);
    // (max constraint degree, constraint count) under the U6 public-degree rule
    std::pair<int, int> stats(int public_degree) const;
    uint32_t log_quotient_degree(int public_degree) const;
    // concrete evaluation folded into acc (verifier / tests)
    void eval_fold(const Fr* loc, const Fr* nxt, const Fr& ap, const Fr& dl, const Fr& first, const Fr& last,
                   const Fr& trans, const Fr& alpha, Fr& acc) const;
};

struct lsp_query {
    std::vector<Fr> trow, tpath, qrow, qpath, sib;
    std::vector<std::vector<Fr>> fpath;
};

}  // namespace lsp

struct lsp_proof {
    uint32_t log_h = 0, log_q = 0, w = 0;
    lsp::Fr troot, qroot, pow_w;
    std::vector<lsp::Fr> tl, tn, qc, roots, final_poly;
    std::vector<lsp::lsp_query> queries;
    // made under a rehearsal transport (lsp_ctx_attach_loopback): peers' data
    // fabricated, so not a proof -- serialize / view refuse it (shape queries only)
    bool rehearsal = false;
    // caches filled on first use by calls that take a const proof (a proof may
    // be shared across threads, e.g. rayon tasks): built under cache_mu
    mutable std::mutex cache_mu;
    mutable std::vector<uint8_t> wire;  // serialize() result, cached by lsp_proof_serialize
    mutable std::shared_ptr<void> view_cache;  // flat arrays behind lsp_proof_view (proof.cpp)
};

// a parsed CBOR RawPermutationTrace / RawLookupTrace (cbor.cpp)
struct lsp_raw_trace {
    int kind = 0;  // LSP_AIR_PERMUTATION or LSP_AIR_LOOKUP
    std::string name;
    std::vector<std::vector<lsp::Fr>> a, b;  // lookup: b = the tables' columns, table-major
    uint32_t ntables = 0, nbc = 0;           // permutation: ntables = number of b columns
    std::vector<lsp::Fr> a_filter;
    std::vector<std::vector<lsp::Fr>> b_filter;
};

struct lsp_tree {
    lsp_ctx* ctx = nullptr;
    size_t height = 0;
    std::vector<size_t> widths;
    lsp::Fr* layers = nullptr;         // device, 2*height - 1
    std::vector<lsp::Fr*> mats;        // device copies (owned) of the committed matrices
};

namespace lsp {
struct Comm;

// Small persistent host thread pool: parallel_for over [0, n) with the
// calling thread participating.  Used for the Merkle tree tops the prover
// finishes on the host: 7 back-to-back levels of a few dozen permutations,
// so a dispatch must cost microseconds, not a condition-variable wake-up per
// level -- workers spin on the job generation for a short window after each
// job (kSpinUs) before sleeping, and the caller spins for completion.
class HostPool {
  public:
    explicit HostPool(unsigned workers);
    ~HostPool();
    void parallel_for(size_t n, const std::function<void(size_t)>& f);
    // get the workers spinning (they spin kSpinUs for the next job) ahead of a
    // parallel_for whose data is about to arrive: no condition-variable wake-up
    // on the critical path.  spin_us > 0: keep spinning until at least that many
    // microseconds from now (cores that slept through a long GPU phase run the
    // next parallel_for slower until they have been busy for a while)
    void wake(unsigned spin_us = 0);
    unsigned size() const { return (unsigned)th_.size() + 1; }
    static constexpr int kSpinUs = 300;

  private:
    void loop();
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_;
    const std::function<void(size_t)>* job_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    std::atomic<unsigned> busy_{0};
    std::atomic<unsigned> sleepers_{0};
    std::atomic<uint64_t> gen_{0};
    std::atomic<bool> stop_{false};
    std::atomic<int64_t> spin_until_ns_{0};  // steady_clock; wake(spin_us)
};
// threads of a context's host pool (the caller included): see host.cpp
unsigned default_host_threads();
}  // namespace lsp

struct lsp_ctx {
    int device = 0;
    lsp::Comm* comm = nullptr;  // attached communicator of a process-per-GPU sharded prove (owned)
    std::unique_ptr<lsp::HostPool> pool_;  // lazily created (host_pool())
    size_t host_tree_top = 1024;            // Merkle levels at or below this many digests run on the host (16 threads, 16-lane IFMA: ~20 us for the 1024 -> 512 level vs ~58 us on the GPU; 1024 beat 256 by ~0.45 ms per 2^19 proof in interleaved same-box runs)
    hipStream_t stream = nullptr;
    lsp::P2Host p2;
    lsp::Fr* rc_dev = nullptr;    // round constants, ark form
    lsp::F29* rc29_dev = nullptr; // the same in the 29-bit-limb form the hash kernels use
    uint32_t log_blowup = 3, log_final_poly_len = 0, num_queries = 33, pow_bits = 0;
    size_t lds_per_block = 64 * 1024;  // the device's LDS per workgroup (hipDeviceAttributeMaxSharedMemoryPerBlock)
    int32_t public_degree = 1;
    lsp::TranscriptCfg transcript;  // U7/U8/U12 (lsp_params)
    std::string err;
    std::mutex mu;
    struct Buf {
        void* p = nullptr;
        size_t cap = 0;
    };
    std::map<std::string, Buf> pool;
    std::map<std::string, Buf> hpool;  // pinned host staging buffers (hbuf)
    std::map<std::string, hipEvent_t> stage_ev;  // last copy out of each h2d_async staging buffer
    hipEvent_t ev_near = nullptr, ev_top = nullptr;  // tree-top hand-off (prove.cpp commit_device)
    hipEvent_t ev_warm = nullptr;  // after a tree's wide levels: the host pool starts spinning (commit_device)
    // work beside a tree's narrow levels (prove.cpp, "constraints before alpha"):
    // a low-priority stream, the event after the tree's wide levels it waits
    // for, and the event the main stream waits for before using its results
    hipStream_t side_stream = nullptr;
    hipEvent_t ev_wide = nullptr, ev_side = nullptr;
    hipStream_t side();  // side_stream, created on first use
    std::vector<hipEvent_t> event_pool;               // phase-timer events, reused across proofs
    // per-phase device timings of lsp_prove (lsp_last_timings): two events per
    // phase, ~0.3 ms of host API time per 2^19 proof; lsp_ctx_set_phase_timing
    // (off, or only the named phases)
    bool phase_timing = true;
    std::vector<std::string> phase_only;
    std::map<std::pair<uint32_t, int>, uint4*> twiddles;
    std::map<std::string, const lsp::Fr*> ptabs;  // cached power tables (prove.cpp pow_table), pool-owned
    // Inside lsp_prove the host-made tree-top layers are only read by the query
    // gather at the end, so their uploads wait there instead of delaying the next
    // kernel on the stream (prove.cpp commit_device / flush_top_uploads).
    struct TopUpload {
        void* dst;
        const void* src;
        size_t bytes;
    };
    bool defer_top_uploads = false;
    std::vector<TopUpload> top_uploads;
    std::map<uint32_t, std::vector<lsp::Fr>> fold_tw;  // host FRI fold factors g^-bitrev(i) per log2 length (prove.cpp)
    size_t fri_host_tail = 2048;  // FRI rounds of at most this many leaves run wholly on the host (prove.cpp)
    std::vector<std::pair<std::string, double>> timings;
    // the last proof's phase events, turned into `timings` lazily
    // (resolve_timings): while the next proof sleeps through its first wide
    // Merkle levels, or when lsp_last_timings asks -- not on the proof's tail
    std::vector<std::tuple<std::string, hipEvent_t, hipEvent_t>> pending_timings;
    // the last proof's data-shaped spans in the reference's bench.log wording
    // (prove.cpp; lsp_last_spans)
    std::vector<std::string> spans;

    void* buf(const std::string& name, size_t bytes);
    lsp::Fr* fbuf(const std::string& name, size_t n) { return (lsp::Fr*)buf(name, n * sizeof(lsp::Fr)); }
    // drain the stream and free every pooled buffer whose name starts with `prefix`
    void release(const std::string& prefix);
    // scratch of a hierarchical batch inverse of n elements (launch_batch_inverse)
    lsp::Fr* bi_scratch(size_t n) { return fbuf("bi_scratch", lsp::batch_inverse_scratch(n) + 1); }
    // pinned host memory; growing it first drains the stream (a copy may still read it)
    // pinned host staging buffer `name`, grown on demand; flags: hipHostMalloc
    // flags (hipHostMallocCoherent for buffers kernels write into directly)
    void* hbuf(const std::string& name, size_t bytes, unsigned flags = 0);
    // asynchronous upload of a small host array through the pinned staging
    // buffer `name`: the caller's memory may be reused at return and the
    // stream is not drained (only the previous copy out of `name` is awaited)
    void h2d_async(const std::string& name, void* dst, const void* src, size_t bytes);
    // w_H^x (or its inverse) for x < H/2, in the 29-bit Montgomery form the NTT multiplies by (k_ntt.hip)
    const uint4* twiddle29(uint32_t logH, bool inverse);
    lsp::HostPool& host_pool();
    void sync();
};
