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
#include "k_common.hpp"
#include "kernels.hpp"
#include "poseidon2_f29.hpp"

namespace lsp {

namespace {
template <uint32_t D>
__global__ __launch_bounds__(256) void k_permute(Fr* __restrict__ st, size_t n, const F29* __restrict__ rc,
                                                 uint32_t rf, uint32_t rp) {
    const size_t i = gtid();
    if (i >= n) return;
    F29 s0 = f29_from_fr(st[3 * i]), s1 = f29_from_fr(st[3 * i + 1]), s2 = f29_from_fr(st[3 * i + 2]);
    permute3_f29<D>(s0, s1, s2, rc, rf, rp);
    st[3 * i] = f29_to_fr(s0);
    st[3 * i + 1] = f29_to_fr(s1);
    st[3 * i + 2] = f29_to_fr(s2);
}

template <uint32_t D>
__global__ __launch_bounds__(256) void k_hash_rows1(const Fr* __restrict__ m, uint32_t w, size_t nrows,
                                                    Fr* __restrict__ out, const F29* __restrict__ rc, uint32_t rf,
                                                    uint32_t rp) {
    const size_t i = gtid();
    if (i >= nrows) return;
    const Fr* row = m + i * w;
    out[i] = sponge_f29<D>([&](uint32_t k) { return row[k]; }, w, rc, rf, rp);
}

template <uint32_t D>
__global__ __launch_bounds__(256) void k_hash_rows_multi(MatList ml, size_t nrows, Fr* __restrict__ out,
                                                         const F29* __restrict__ rc, uint32_t rf, uint32_t rp) {
    const size_t i = gtid();
    if (i >= nrows) return;
    uint32_t total = 0;
    for (uint32_t j = 0; j < ml.n; ++j) total += ml.width[j];
    auto get = [&](uint32_t k) {
        uint32_t j = 0;
        while (k >= ml.width[j]) {
            k -= ml.width[j];
            ++j;
        }
        return ml.ptr[j][i * ml.width[j] + k];
    };
    out[i] = sponge_f29<D>(get, total, rc, rf, rp);
}

template <uint32_t D>
__global__ __launch_bounds__(256) void k_merkle_level(const Fr* __restrict__ src, Fr* __restrict__ dst, size_t nout,
                                                      const F29* __restrict__ rc, uint32_t rf, uint32_t rp) {
    const size_t i = gtid();
    if (i >= nout) return;
    dst[i] = compress_f29<D>(src[2 * i], src[2 * i + 1], rc, rf, rp);
}

// Top of a tree in one workgroup: `len` (<= 2*blockDim, power of two) digests at
// layers[off..off+len) -> every layer above them, through the LDS.
template <uint32_t D>
__global__ __launch_bounds__(64) void k_merkle_top(Fr* __restrict__ layers, size_t off, uint32_t len,
                                                    const F29* __restrict__ rc, uint32_t rf, uint32_t rp) {
    __shared__ Fr buf[128];
    for (uint32_t e = threadIdx.x; e < len; e += blockDim.x) buf[e] = layers[off + e];
    __syncthreads();
    size_t out_off = off + len;
    while (len > 1) {
        const uint32_t nout = len / 2;
        Fr r;
        if (threadIdx.x < nout) r = compress_f29<D>(buf[2 * threadIdx.x], buf[2 * threadIdx.x + 1], rc, rf, rp);
        __syncthreads();
        if (threadIdx.x < nout) {
            buf[threadIdx.x] = r;
            layers[out_off + threadIdx.x] = r;
        }
        __syncthreads();
        out_off += nout;
        len = nout;
    }
}
// PoW grinding (GrindingChallenger::grind, [EXT p3-challenger]; U8): each lane
// tests candidate witnesses w: the sponge state before the block holding w is
// fixed (host), w is absorbed into lane `wlane` (the other rate lane keeps
// `other`), one permutation, then the low `bits` of the canonical s0 must be 0.
// The smallest hit of the batch is kept with an atomic min.
template <uint32_t D>
__global__ __launch_bounds__(256) void k_grind(Fr pre0, Fr pre1, Fr pre2, uint32_t wlane, uint64_t base,
                                               uint64_t count, uint32_t bits, const F29* __restrict__ rc,
                                               uint32_t rf, uint32_t rp, unsigned long long* __restrict__ best) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const F29 c0 = f29_from_fr(pre0), c1 = f29_from_fr(pre1), c2 = f29_from_fr(pre2);
    const uint64_t mask = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
    for (uint64_t i = gtid(); i < count; i += stride) {
        const uint64_t w = base + i;
        const F29 fw = f29_from_fr(fr_from_u64(w));
        F29 s0 = wlane == 0 ? fw : c0, s1 = wlane == 0 ? c1 : fw, s2 = c2;
        permute3_f29<D>(s0, s1, s2, rc, rf, rp);
        const Fr c = fr_to_canonical(f29_to_fr(s0));
        const uint64_t lo = (uint64_t)c.v[0] | ((uint64_t)c.v[1] << 32);
        if ((lo & mask) == 0) atomicMin(best, (unsigned long long)w);
    }
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

#define LSP_DISPATCH_D(L, KERNEL, ...)                                  \
    do {                                                                \
        if ((L).sbox_degree == 17)                                      \
            hipLaunchKernelGGL(KERNEL<17>, __VA_ARGS__);                \
        else                                                            \
            hipLaunchKernelGGL(KERNEL<11>, __VA_ARGS__);                \
    } while (0)

hipError_t launch_permute(Fr* states, size_t n, const F29* rc, P2Layout L, hipStream_t st) {
    if (!n) return hipSuccess;
    LSP_DISPATCH_D(L, k_permute, dim3(nblocks(n, 256)), dim3(256), 0, st, states, n, rc, L.rounds_f, L.rounds_p);
    return hipGetLastError();
}

hipError_t launch_hash_rows(const MatList& m, size_t nrows, Fr* out, const F29* rc, P2Layout L, hipStream_t st) {
    if (!nrows) return hipSuccess;
    const unsigned bs = nrows >= (1u << 14) ? 256u : 64u;  // spread narrow batches over more CUs
    if (m.n == 1)
        LSP_DISPATCH_D(L, k_hash_rows1, dim3(nblocks(nrows, bs)), dim3(bs), 0, st, m.ptr[0], m.width[0], nrows,
                       out, rc, L.rounds_f, L.rounds_p);
    else
        LSP_DISPATCH_D(L, k_hash_rows_multi, dim3(nblocks(nrows, bs)), dim3(bs), 0, st, m, nrows, out, rc,
                       L.rounds_f, L.rounds_p);
    return hipGetLastError();
}

hipError_t launch_grind(const Fr pre[3], uint32_t wlane, uint64_t base, uint64_t count, uint32_t bits,
                        const F29* rc, P2Layout L, unsigned long long* best, hipStream_t st) {
    const unsigned blocks = 256 * 16;
    LSP_DISPATCH_D(L, k_grind, dim3(blocks), dim3(256), 0, st, pre[0], pre[1], pre[2], wlane, base, count, bits, rc,
                   L.rounds_f, L.rounds_p, best);
    return hipGetLastError();
}

hipError_t launch_merkle_level(const Fr* src, Fr* dst, size_t nout, const F29* rc, P2Layout L, hipStream_t st) {
    if (!nout) return hipSuccess;
    LSP_DISPATCH_D(L, k_merkle_level, dim3(nblocks(nout, 256)), dim3(256), 0, st, src, dst, nout, rc, L.rounds_f,
                   L.rounds_p);
    return hipGetLastError();
}

hipError_t launch_merkle_tree(Fr* layers, size_t nleaves, const F29* rc, P2Layout L, hipStream_t st) {
    // Wide levels: one compression per lane, 256-lane blocks.  Narrow levels
    // (< 2^14 nodes) are latency-bound (one permutation per level on the
    // critical path): 64-lane blocks spread their waves over as many CUs as
    // possible.  The last 64 -> 1 levels run in one wave.
    size_t off = 0, len = nleaves;
    while (len > 64) {
        const size_t nout = len / 2;
        const unsigned bs = nout >= (1u << 14) ? 256u : 64u;
        LSP_DISPATCH_D(L, k_merkle_level, dim3(nblocks(nout, bs)), dim3(bs), 0, st, layers + off, layers + off + len,
                       nout, rc, L.rounds_f, L.rounds_p);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        off += len;
        len /= 2;
    }
    if (len > 1) {
        LSP_DISPATCH_D(L, k_merkle_top, dim3(1), dim3(64), 0, st, layers, off, (uint32_t)len, rc, L.rounds_f,
                       L.rounds_p);
        return hipGetLastError();
    }
    return hipSuccess;
}

}  // namespace lsp
