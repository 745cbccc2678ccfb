// Poseidon2-w3 permutation batches, row hashing (PaddingFreeSponge) and
// Merkle levels (CompressionFunctionFromHasher) -- the kernels behind
// MerkleTreeMmcs::commit ([EXT p3-merkle-tree], bin/src/config.rs:19-20).
//
// One thread owns one permutation state; the work is integer VALU bound
// (~230 Montgomery products per permutation), so the kernels are plain
// one-state-per-lane loops with the round constants on the scalar path
// (uniform addresses -> s_load).  The permutation runs on the 29-bit-limb
// representation (fr29.hpp / poseidon2_f29.hpp: carry-free 64-bit column
// accumulation, 1.34x the 32-bit-limb permutation rate on MI355X); inputs and
// digests stay in the ark-ff form.
#include <cstdlib>

#include "k_common.hpp"
#include "kernels.hpp"
#include "poseidon2_f29.hpp"
#include "poseidon2_row.hpp"

namespace lsp {

// waves per SIMD requested for the one-row-per-lane leaf kernels (the LDS
// reduction table lets the compiler hoist loads and grow to 3 waves)
#ifndef LSP_P2_ROWS_WPE
#define LSP_P2_ROWS_WPE 1
#endif

namespace {
template <uint32_t D>
__global__ __launch_bounds__(256) void k_permute(Fr* __restrict__ st, size_t n, const F29* __restrict__ rc,
                                                 uint32_t rf, uint32_t rp) {
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt's table
    f29_qtab_init(qt);
    __syncthreads();
    const size_t i = gtid();
    if (i >= n) return;
    F29 s0 = f29_from_fr(st[3 * i]), s1 = f29_from_fr(st[3 * i + 1]), s2 = f29_from_fr(st[3 * i + 2]);
    permute3_any<D, 1>(s0, s1, s2, rc, rf, rp, qt);
    st[3 * i] = f29_to_fr(s0);
    st[3 * i + 1] = f29_to_fr(s1);
    st[3 * i + 2] = f29_to_fr(s2);
}

// LANES: lanes per row -- 4 (a DPP quad) or 2 (a pair) for batches narrower
// than the chip (poseidon2_f29.hpp), otherwise 1.
template <uint32_t D, int LANES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LSP_P2_ROWS_WPE))) void k_hash_rows1(const Fr* __restrict__ m, uint32_t w, size_t nrows,
                                                    Fr* __restrict__ out, const F29* __restrict__ rc, uint32_t rf,
                                                    uint32_t rp) {
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt's table
    f29_qtab_init(qt);
    __syncthreads();
    const size_t i = gtid() / LANES;
    if (i >= nrows) return;
    const Fr* row = m + i * w;
    const Fr d = sponge_f29<D, LANES>([&](uint32_t k) { return LSP_BOUNDS(k < w) ? row[k] : fr_zero(); }, w, rc, rf,
                                      rp, qt);
    if ((threadIdx.x & (LANES - 1)) == 0) out[i] = d;
}

template <uint32_t D, int LANES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LSP_P2_ROWS_WPE))) void k_hash_rows_multi(MatList ml, size_t nrows, Fr* __restrict__ out,
                                                         const F29* __restrict__ rc, uint32_t rf, uint32_t rp) {
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt's table
    f29_qtab_init(qt);
    __syncthreads();
    const size_t i = gtid() / LANES;
    if (i >= nrows) return;
    uint32_t total = 0;
    for (uint32_t j = 0; j < ml.n; ++j) total += ml.width[j];
    auto get = [&](uint32_t k) {
        uint32_t j = 0;
        while (k >= ml.width[j]) {
            k -= ml.width[j];
            ++j;
            if (!LSP_BOUNDS(j < ml.n)) return fr_zero();
        }
        return ml.ptr[j][i * ml.width[j] + k];
    };
    const Fr d = sponge_f29<D, LANES>(get, total, rc, rf, rp, qt);
    if ((threadIdx.x & (LANES - 1)) == 0) out[i] = d;
}

template <uint32_t D, int LANES>
__global__ __launch_bounds__(256) void k_fold_hash(FoldSpec f, size_t nleaves, Fr* __restrict__ out,
                                                   const F29* __restrict__ rc, uint32_t rf, uint32_t rp) {
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt's table
    f29_qtab_init(qt);
    __syncthreads();
    const size_t j = gtid() / LANES;
    if (j >= nleaves) return;
    Fr e[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const size_t i = 2 * j + k;
        const Fr p = fr_mul(f.half_beta, pow2l(f.tab, f.L1, brev_bits(f.i0 + i, f.logm)));
        e[k] = fr_add(fr_mul(fr_add(f.half, p), f.v[2 * i]), fr_mul(fr_sub(f.half, p), f.v[2 * i + 1]));
    }
    if ((threadIdx.x & (LANES - 1)) == 0) {
        f.vout[2 * j] = e[0];
        f.vout[2 * j + 1] = e[1];
    }
    const Fr d = sponge_f29<D, LANES>([&](uint32_t k) { return e[k]; }, 2, rc, rf, rp, qt);
    if ((threadIdx.x & (LANES - 1)) == 0) out[j] = d;
}

template <uint32_t D, int LANES>
__global__ __launch_bounds__(256) void k_merkle_level(const Fr* __restrict__ src, Fr* __restrict__ dst, size_t nout,
                                                      const F29* __restrict__ rc, uint32_t rf, uint32_t rp) {
    // the narrow forms are one permutation's latency per level, the critical
    // path: their waves win the SIMD's issue arbitration against work a side
    // stream runs beside them (prove.cpp, constraints before alpha)
    if constexpr (LANES > 1) __builtin_amdgcn_s_setprio(3);
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt's table
    f29_qtab_init(qt);
    __syncthreads();
    const size_t i = gtid() / LANES;
    if (i >= nout) return;
    if (!LSP_BOUNDS(2 * i + 1 < 2 * nout)) return;
    const Fr d = compress_f29<D, LANES>(src[2 * i], src[2 * i + 1], rc, rf, rp, qt);
    if ((threadIdx.x & (LANES - 1)) == 0) dst[i] = d;
}

// The narrowest levels (nout <= row_max(), default linear layers): one node per
// wave, the state spread over the lanes (poseidon2_row.hpp) -- the level is one
// compression's single-wave latency, which the 16-lane row product shortens
template <uint32_t D>
__global__ __launch_bounds__(64) void k_merkle_level_row(const Fr* __restrict__ src, Fr* __restrict__ dst,
                                                         size_t nout, const F29* __restrict__ rc, uint32_t rf,
                                                         uint32_t rp) {
    __builtin_amdgcn_s_setprio(3);
    __shared__ prow::RowLds tab;
    prow::row_lds_init(&tab);
    __syncthreads();
    const size_t i = blockIdx.x;
    if (i >= nout) return;
    const Fr d = prow::compress_row<D>(src + 2 * i, src + 2 * i + 1, rc, rf, rp, &tab);
    if (threadIdx.x == 0) dst[i] = d;
}

// Top of a tree in one workgroup of 4 * 64 lanes: `len` (<= 128, power of
// two) digests at layers[off..off+len) -> every layer above them, one
// compression per DPP quad, through the LDS.
template <uint32_t D>
__global__ __launch_bounds__(256) void k_merkle_top(Fr* __restrict__ layers, size_t off, uint32_t len,
                                                    const F29* __restrict__ rc, uint32_t rf, uint32_t rp) {
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt's table
    f29_qtab_init(qt);
    __syncthreads();
    __shared__ Fr buf[128];
    if (!LSP_BOUNDS(len <= 128)) return;
    for (uint32_t e = threadIdx.x; e < len; e += blockDim.x) buf[e] = layers[off + e];
    __syncthreads();
    size_t out_off = off + len;
    const uint32_t q = threadIdx.x >> 2;
    const bool lead = (threadIdx.x & 3) == 0;
    while (len > 1) {
        const uint32_t nout = len / 2;
        Fr r;
        if (q < nout) r = compress_f29<D, 4>(buf[2 * q], buf[2 * q + 1], rc, rf, rp, qt);
        __syncthreads();
        if (q < nout && lead) {
            buf[q] = r;
            layers[out_off + q] = r;
        }
        __syncthreads();
        out_off += nout;
        len = nout;
    }
}
// PoW grinding (GrindingChallenger::grind, [EXT p3-challenger]; U8): each lane
// tests candidate witnesses w: the sponge state before the block holding w is
// fixed (host), w is absorbed into lane `wlane` (the other rate lane keeps
// `other`), one permutation, then the low `bits` of the canonical s0 (mont:
// of its Montgomery form, U8's switch) must be 0.
// The smallest hit of the batch is kept with an atomic min.
template <uint32_t D>
__global__ __launch_bounds__(256) void k_grind(Fr pre0, Fr pre1, Fr pre2, uint32_t wlane, uint64_t base,
                                               uint64_t count, uint32_t bits, uint32_t mont, const F29* __restrict__ rc,
                                               uint32_t rf, uint32_t rp, unsigned long long* __restrict__ best) {
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt's table
    f29_qtab_init(qt);
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const F29 c0 = f29_from_fr(pre0), c1 = f29_from_fr(pre1), c2 = f29_from_fr(pre2);
    const uint64_t mask = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
    for (uint64_t i = gtid(); i < count; i += stride) {
        const uint64_t w = base + i;
        const F29 fw = f29_from_fr(fr_from_u64(w));
        F29 s0 = wlane == 0 ? fw : c0, s1 = wlane == 0 ? c1 : fw, s2 = c2;
        permute3_any<D, 1>(s0, s1, s2, rc, rf, rp, qt);
        const Fr m = f29_to_fr(s0);  // Montgomery form, reduced
        const Fr c = mont ? m : fr_to_canonical(m);
        const uint64_t lo = (uint64_t)c.v[0] | ((uint64_t)c.v[1] << 32);
        if ((lo & mask) == 0) atomicMin(best, (unsigned long long)w);
    }
}

// Permutation-throughput probe (the peak the Merkle kernels are quoted
// against): `iters` chained permutations per lane on register-resident states.
template <uint32_t D>
__global__ __launch_bounds__(256) void k_calib_perm(Fr* __restrict__ out, uint32_t iters, const F29* __restrict__ rc,
                                                    uint32_t rf, uint32_t rp) {
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt's table
    f29_qtab_init(qt);
    __syncthreads();
    const size_t t = gtid();
    F29 s0 = f29_from_fr(fr_from_u64(t + 1)), s1 = f29_from_fr(fr_from_u64(3 * t + 7)), s2 = f29_zero();
    for (uint32_t i = 0; i < iters; ++i) permute3_any<D, 1>(s0, s1, s2, rc, rf, rp, qt);
    out[t] = f29_to_fr(s0);
}

__global__ void k_rc_to_f29(const Fr* __restrict__ rc, F29* __restrict__ rc29, uint32_t n) {
    const uint32_t i = (uint32_t)gtid();
    if (i < n) rc29[i] = f29_from_fr(rc[i]);
}
}  // namespace

hipError_t launch_rc_to_f29(const Fr* rc, F29* rc29, uint32_t n, hipStream_t st) {
    hipLaunchKernelGGL(k_rc_to_f29, dim3(nblocks(n, 64)), dim3(64), 0, st, rc, rc29, n);
    return hipGetLastError();
}

// D = the S-box degree, | P2_GEN for caller-set linear layers (gen_lin)
#define LSP_DISPATCH_D(L, KERNEL, ...)                                  \
    do {                                                                \
        if ((L).gen_lin) {                                              \
            if ((L).sbox_degree == 17)                                  \
                hipLaunchKernelGGL(KERNEL<17u | P2_GEN>, __VA_ARGS__);  \
            else                                                        \
                hipLaunchKernelGGL(KERNEL<11u | P2_GEN>, __VA_ARGS__);  \
        } else if ((L).sbox_degree == 17)                               \
            hipLaunchKernelGGL(KERNEL<17>, __VA_ARGS__);                \
        else                                                            \
            hipLaunchKernelGGL(KERNEL<11>, __VA_ARGS__);                \
    } while (0)

// (degree, lanes) dispatch.  A batch of at most COOP_MAX permutations runs one
// state per DPP quad: 4 * COOP_MAX lanes = one wave per SIMD of the 256 CUs,
// where the quad form's shorter critical path (30 vs 46 S-boxes) wins; wider
// batches are throughput-bound and keep one state per lane.
#define LSP_DISPATCH_DL(DEG, LANES, KERNEL, ...)                          \
    do {                                                                  \
        if ((LANES) == 4)                                                 \
            hipLaunchKernelGGL((KERNEL<DEG, 4>), __VA_ARGS__);            \
        else if ((LANES) == 2)                                            \
            hipLaunchKernelGGL((KERNEL<DEG, 2>), __VA_ARGS__);            \
        else                                                              \
            hipLaunchKernelGGL((KERNEL<DEG, 1>), __VA_ARGS__);            \
    } while (0)
#define LSP_DISPATCH_DC(L, LANES, KERNEL, ...)                            \
    do {                                                                  \
        if ((L).gen_lin) {                                                \
            if ((L).sbox_degree == 17)                                    \
                LSP_DISPATCH_DL(17u | P2_GEN, LANES, KERNEL, __VA_ARGS__);\
            else                                                          \
                LSP_DISPATCH_DL(11u | P2_GEN, LANES, KERNEL, __VA_ARGS__);\
        } else if ((L).sbox_degree == 17)                                 \
            LSP_DISPATCH_DL(17u, LANES, KERNEL, __VA_ARGS__);             \
        else                                                              \
            LSP_DISPATCH_DL(11u, LANES, KERNEL, __VA_ARGS__);             \
    } while (0)

static size_t coop_max() {
    static const size_t v = [] {
        const char* e = std::getenv("LSP_COOP_MAX");
        return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)16384;
    }();
    return v;
}
static unsigned coop_bs() {  // 0: by width (state_grid)
    static const unsigned v = [] {
        const char* e = std::getenv("LSP_COOP_BS");
        return e ? (unsigned)std::strtoul(e, nullptr, 10) : 0u;
    }();
    return v;
}
#define COOP_MAX coop_max()
// up to this many states a pair per state (2 lanes): at 32K states one wave per
// SIMD with 168 instead of 230 products on each lane's critical path
static size_t pair_max() {
    static const size_t v = [] {
        const char* e = std::getenv("LSP_PAIR_MAX");
        return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)32768;
    }();
    return v;
}
static inline int lanes_for(size_t n) { return n <= COOP_MAX ? 4 : (n <= pair_max() ? 2 : 1); }

// grid for n states: quads in 64-lane blocks (256 from 16K states: one wave
// per SIMD), pairs and single lanes in 256-lane blocks
static inline void state_grid(size_t n, int lanes, unsigned& blocks, unsigned& bs) {
    if (lanes == 4) {
        // 4 lanes per state.  At 16K states (one wave per SIMD of the chip) 64-lane
        // blocks land two waves on some SIMDs (~2x the level's latency); 256-lane
        // blocks, one per CU, spread them one per SIMD.  Narrower levels: 64.
        bs = coop_bs() ? coop_bs() : (4 * n >= 65536 ? 256u : 64u);
        blocks = nblocks(4 * n, bs);
    } else {
        bs = 256;
        blocks = nblocks((size_t)lanes * n, bs);
    }
}

hipError_t launch_permute(Fr* states, size_t n, const F29* rc, P2Layout L, hipStream_t st) {
    if (!n) return hipSuccess;
    LSP_DISPATCH_D(L, k_permute, dim3(nblocks(n, 256)), dim3(256), 0, st, states, n, rc, L.rounds_f, L.rounds_p);
    return hipGetLastError();
}

hipError_t launch_hash_rows(const MatList& m, size_t nrows, Fr* out, const F29* rc, P2Layout L, hipStream_t st) {
    if (!nrows) return hipSuccess;
    const int lanes = lanes_for(nrows);
    unsigned blocks, bs;
    state_grid(nrows, lanes, blocks, bs);
    if (m.n == 1)
        LSP_DISPATCH_DC(L, lanes, k_hash_rows1, dim3(blocks), dim3(bs), 0, st, m.ptr[0], m.width[0], nrows, out, rc,
                        L.rounds_f, L.rounds_p);
    else
        LSP_DISPATCH_DC(L, lanes, k_hash_rows_multi, dim3(blocks), dim3(bs), 0, st, m, nrows, out, rc, L.rounds_f,
                        L.rounds_p);
    return hipGetLastError();
}

hipError_t launch_fold_hash(const FoldSpec& f, size_t nleaves, Fr* out, const F29* rc, P2Layout L, hipStream_t st) {
    if (!nleaves) return hipSuccess;
    const int lanes = lanes_for(nleaves);
    unsigned blocks, bs;
    state_grid(nleaves, lanes, blocks, bs);
    LSP_DISPATCH_DC(L, lanes, k_fold_hash, dim3(blocks), dim3(bs), 0, st, f, nleaves, out, rc, L.rounds_f, L.rounds_p);
    return hipGetLastError();
}

hipError_t launch_calib_perm(Fr* out, size_t nthreads, uint32_t iters, const F29* rc, P2Layout L, hipStream_t st) {
    LSP_DISPATCH_D(L, k_calib_perm, dim3(nblocks(nthreads, 256)), dim3(256), 0, st, out, iters, rc, L.rounds_f,
                   L.rounds_p);
    return hipGetLastError();
}

hipError_t launch_grind(const Fr pre[3], uint32_t wlane, uint64_t base, uint64_t count, uint32_t bits, bool mont,
                        const F29* rc, P2Layout L, unsigned long long* best, hipStream_t st) {
    const unsigned blocks = 256 * 16;
    LSP_DISPATCH_D(L, k_grind, dim3(blocks), dim3(256), 0, st, pre[0], pre[1], pre[2], wlane, base, count, bits,
                   (uint32_t)mont, rc,
                   L.rounds_f, L.rounds_p, best);
    return hipGetLastError();
}

// levels of at most this many nodes run the row form (k_merkle_level_row);
// LSP_ROW_MAX=0 keeps the quad form
static size_t row_max() {
    static const size_t v = [] {
        const char* e = std::getenv("LSP_ROW_MAX");
        return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)1024;
    }();
    return v;
}

hipError_t launch_merkle_level(const Fr* src, Fr* dst, size_t nout, const F29* rc, P2Layout L, hipStream_t st) {
    if (!nout) return hipSuccess;
    if (!L.gen_lin && nout <= row_max()) {
        if (L.sbox_degree == 17)
            hipLaunchKernelGGL(k_merkle_level_row<17>, dim3((unsigned)nout), dim3(64), 0, st, src, dst, nout, rc,
                               L.rounds_f, L.rounds_p);
        else
            hipLaunchKernelGGL(k_merkle_level_row<11>, dim3((unsigned)nout), dim3(64), 0, st, src, dst, nout, rc,
                               L.rounds_f, L.rounds_p);
        return hipGetLastError();
    }
    const int lanes = lanes_for(nout);
    unsigned blocks, bs;
    state_grid(nout, lanes, blocks, bs);
    LSP_DISPATCH_DC(L, lanes, k_merkle_level, dim3(blocks), dim3(bs), 0, st, src, dst, nout, rc, L.rounds_f,
                    L.rounds_p);
    return hipGetLastError();
}

hipError_t launch_merkle_levels(Fr* layers, size_t nleaves, size_t stop_len, const F29* rc, P2Layout L,
                                size_t* off_out, size_t* len_out, hipStream_t st) {
    size_t off = 0, len = nleaves;
    while (len > stop_len && len > 1) {
        hipError_t e = launch_merkle_level(layers + off, layers + off + len, len / 2, rc, L, st);
        if (e != hipSuccess) return e;
        off += len;
        len /= 2;
    }
    *off_out = off;
    *len_out = len;
    return hipSuccess;
}

hipError_t launch_merkle_tree(Fr* layers, size_t nleaves, const F29* rc, P2Layout L, hipStream_t st) {
    // One launch per level down to 128 digests (launch_merkle_level picks the
    // per-lane or per-quad form by width), then the last 128 -> 1 levels in
    // one workgroup.
    size_t off = 0, len = nleaves;
    while (len > 128) {
        const size_t nout = len / 2;
        hipError_t e = launch_merkle_level(layers + off, layers + off + len, nout, rc, L, st);
        if (e != hipSuccess) return e;
        off += len;
        len /= 2;
    }
    if (len > 1) {
        LSP_DISPATCH_D(L, k_merkle_top, dim3(1), dim3(256), 0, st, layers, off, (uint32_t)len, rc, L.rounds_f,
                       L.rounds_p);
        return hipGetLastError();
    }
    return hipSuccess;
}

}  // namespace lsp

LSP_BOUNDS_READER(k_hash)
