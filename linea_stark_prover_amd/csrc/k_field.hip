// Batch inversion (p3-field batch_multiplicative_inverse) and the gather used
// to pull query openings off the device in one copy.
#include "fr29.hpp"
#include "k_common.hpp"
#include "kernels.hpp"

namespace lsp {

namespace {
// Batch inversion, hierarchical (Montgomery's trick at every level):
//   up    workgroup b owns the 4096 elements [4096 b, 4096 b + 4096): thread t
//         the 16 elements 4096 b + 256 j + t (every pass coalesced), whose
//         prefix products it writes to out[]; the 256 chunk products go up a
//         product tree in LDS and prod[b] = the workgroup's product;
//   the workgroup products are inverted the same way, recursively, down to a
//   base of <= BI_BASE elements that one workgroup inverts with a product
//   tree in LDS and ONE Fermat inverse (on the 29-bit multiplier) -- skipped
//   when the caller knows the inverse of the whole product;
//   down  workgroup b rebuilds its tree (a thread's chunk product is its last
//         prefix times its last element), takes 1/prod[b] down the tree and
//         walks every chunk backwards.
// Cost ~3 products per element plus one inversion for the whole batch; one
// level per 4096x (2^22 elements: up, base, down -- three launches; the
// per-thread chains of the earlier 16x levels took seven).
constexpr uint32_t BI_THREADS = 256;
constexpr uint32_t BI_CHUNK = 16;
constexpr uint32_t BI_WG = BI_THREADS * BI_CHUNK;  // elements per workgroup of the up/down passes
constexpr uint32_t BI_BASE = BI_THREADS * 16;

// the product tree of a workgroup's 256 chunk products (node k: children 2k,
// 2k+1; leaves at BI_THREADS + t); ends with a barrier
__device__ __forceinline__ void bi_tree_up(Fr* tree, uint32_t t, const Fr& acc) {
    tree[BI_THREADS + t] = acc;
    __syncthreads();
    for (uint32_t w = BI_THREADS / 2; w >= 1; w >>= 1) {
        if (t < w) tree[w + t] = fr_mul(tree[2 * (w + t)], tree[2 * (w + t) + 1]);
        __syncthreads();
    }
}

// tree[1] = 1/(the root's product) on entry; afterwards node k holds 1/(its
// subtree's product), so leaf BI_THREADS + t is 1/(chunk t's product)
__device__ __forceinline__ void bi_tree_down(Fr* tree, uint32_t t) {
    for (uint32_t w = 1; w < BI_THREADS; w <<= 1) {
        Fr l, r;
        if (t < w) {
            const Fr iv = tree[w + t];
            l = fr_mul(iv, tree[2 * (w + t) + 1]);
            r = fr_mul(iv, tree[2 * (w + t)]);
        }
        __syncthreads();
        if (t < w) {
            tree[2 * (w + t)] = l;
            tree[2 * (w + t) + 1] = r;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(BI_THREADS) void k_bi_up(const Fr* __restrict__ in, Fr* __restrict__ out, size_t n,
                                                      Fr* __restrict__ prod) {
    __shared__ Fr tree[2 * BI_THREADS];
    const uint32_t t = threadIdx.x;
    const size_t base = (size_t)blockIdx.x * BI_WG + t;
    Fr acc = fr_one();
    for (uint32_t j = 0; j < BI_CHUNK; ++j) {
        const size_t i = base + (size_t)j * BI_THREADS;
        if (i >= n) break;
        out[i] = acc;
        acc = fr_mul(acc, in[i]);
    }
    bi_tree_up(tree, t, acc);
    if (t == 0) prod[blockIdx.x] = tree[1];
}

__global__ __launch_bounds__(BI_THREADS) void k_bi_down(const Fr* __restrict__ in, Fr* __restrict__ out, size_t n,
                                                        const Fr* __restrict__ inv_prod) {
    __shared__ Fr tree[2 * BI_THREADS];
    const uint32_t t = threadIdx.x;
    const size_t base = (size_t)blockIdx.x * BI_WG + t;
    const uint32_t cnt = base >= n ? 0u : (uint32_t)min((size_t)BI_CHUNK, (n - 1 - base) / BI_THREADS + 1);
    Fr acc = fr_one();
    if (cnt) {
        const size_t il = base + (size_t)(cnt - 1) * BI_THREADS;
        acc = fr_mul(out[il], in[il]);  // the chunk's product: its last prefix times its last element
    }
    bi_tree_up(tree, t, acc);
    if (t == 0) tree[1] = inv_prod[blockIdx.x];
    __syncthreads();
    bi_tree_down(tree, t);
    Fr inv = tree[BI_THREADS + t];
    for (uint32_t j = cnt; j-- > 0;) {
        const size_t i = base + (size_t)j * BI_THREADS;
        const Fr o = fr_mul(inv, out[i]);
        inv = fr_mul(inv, in[i]);
        out[i] = o;
    }
}

// a^(r-2) on the 29-bit multiplier (Fermat; the inverse of zero is zero)
__device__ Fr fr_inv_f29(const Fr& a) {
    const F29 x = f29_from_fr(a);
    F29 r = x;  // the exponent's top bit
    for (int w = 7; w >= 0; --w) {
        // r - 2: r[0] = 1, so the subtraction borrows from word 1
        const uint32_t e = w == 0 ? 0xffffffffu : (w == 1 ? LSP_MOD1 - 1u : mod_word(w));
        const int top = w == 7 ? 31 - __builtin_clz(e) - 1 : 31;
        for (int k = top; k >= 0; --k) {
            r = f29_sqr(r);
            if ((e >> k) & 1u) r = f29_mul(r, x);
        }
    }
    return f29_to_fr(r);
}

// n <= BI_BASE: per-thread chunks (stride BI_THREADS), a product tree over the
// BI_THREADS chunk products in LDS, one inversion, back down the tree
// have_inv: the caller knows 1/(product of all n inputs) (inv_total), e.g. the
// open phase's 1/(zeta^S - c^S) over a coset, and the Fermat inversion -- a
// ~150 us chain of ~380 products on one lane -- is skipped
__global__ __launch_bounds__(BI_THREADS) void k_bi_base(const Fr* __restrict__ in, Fr* __restrict__ out, size_t n,
                                                         Fr inv_total, int have_inv) {
    __shared__ Fr tree[2 * BI_THREADS];  // node k: children 2k, 2k+1; leaves at BI_THREADS + t
    const uint32_t t = threadIdx.x;
    Fr acc = fr_one();
    for (size_t i = t; i < n; i += BI_THREADS) {
        out[i] = acc;
        acc = fr_mul(acc, in[i]);
    }
    bi_tree_up(tree, t, acc);
    if (t == 0) tree[1] = have_inv ? inv_total : fr_inv_f29(tree[1]);
    __syncthreads();
    bi_tree_down(tree, t);
    Fr inv = tree[BI_THREADS + t];
    if (t >= n) return;
    const size_t last = t + ((n - 1 - t) / BI_THREADS) * BI_THREADS;
    for (size_t i = last;; i -= BI_THREADS) {
        const Fr o = fr_mul(inv, out[i]);
        inv = fr_mul(inv, in[i]);
        out[i] = o;
        if (i < BI_THREADS) break;
    }
}

// single-level kernel (no scratch): one Fermat inverse per thread
// Thread t owns elements t, t+T, t+2T, ... (`chunk` of them, interleaved so every
// pass is coalesced): a prefix product, one Fermat inverse, the back pass.  The
// inverse (~380 products) is one instruction stream per wave whatever the
// chunk, so the launcher sizes the chunk for about one wave per SIMD.
__global__ __launch_bounds__(256) void k_batch_inverse(const Fr* __restrict__ in, Fr* __restrict__ out, size_t n,
                                                       size_t T, uint32_t chunk) {
    const size_t t = gtid();
    if (t >= T) return;
    Fr acc = fr_one();
    uint32_t cnt = 0;
    for (uint32_t j = 0; j < chunk; ++j) {
        const size_t i = t + (size_t)j * T;
        if (i >= n) break;
        out[i] = acc;
        acc = fr_mul(acc, in[i]);
        ++cnt;
    }
    Fr inv = fr_inv(acc);
    for (uint32_t j = cnt; j-- > 0;) {
        const size_t i = t + (size_t)j * T;
        const Fr o = fr_mul(inv, out[i]);
        inv = fr_mul(inv, in[i]);
        out[i] = o;
    }
}

// Fr-mul throughput probe of the multiplier the Poseidon2 kernels use (the
// 29-bit-limb product, fr29.hpp): 4 independent register-resident chains per lane
__global__ __launch_bounds__(256) void k_calib_mul(Fr* __restrict__ out, uint32_t iters) {
    const size_t t = gtid();
    F29 a = f29_from_fr(fr_from_u64(t + 3)), b = f29_from_fr(fr_from_u64(t * 7 + 5)),
        c = f29_from_fr(fr_from_u64(t + 11)), d = f29_from_fr(fr_from_u64(t + 13));
    const F29 m = f29_from_fr(fr_from_u64(0x1234567u + (uint32_t)t));
    for (uint32_t i = 0; i < iters; ++i) {
        a = f29_mul(a, m);
        b = f29_mul(b, m);
        c = f29_mul(c, m);
        d = f29_mul(d, m);
    }
    out[t] = fr_add(fr_add(f29_to_fr(a), f29_to_fr(b)), fr_add(f29_to_fr(c), f29_to_fr(d)));
}

__global__ __launch_bounds__(256) void k_gather(const uint64_t* __restrict__ ptrs, Fr* __restrict__ out, size_t n) {
    const size_t i = gtid();
    if (i < n) out[i] = *reinterpret_cast<const Fr*>(ptrs[i]);
}

__global__ __launch_bounds__(256) void k_assemble_chunks(const Fr* __restrict__ stage, uint32_t logGq, size_t Sq,
                                                         Fr* __restrict__ out) {
    const size_t i = gtid();
    if (i >= (Sq << logGq)) return;
    out[i] = stage[brev_bits(i & ((1ull << logGq) - 1), logGq) * Sq + (i >> logGq)];
}
// the debug build's self-test (lsp_debug_bounds_probe): one check that must
// fail, on an index one past its extent; nothing is accessed
__global__ void k_bounds_probe(uint32_t n, uint32_t* __restrict__ sink) {
    const uint32_t i = n + threadIdx.x;  // == n for the one thread
    if (LSP_BOUNDS(i < n)) sink[i] = 1u;
}
}  // namespace

hipError_t launch_bounds_probe(uint32_t* sink, hipStream_t st) {
    hipLaunchKernelGGL(k_bounds_probe, dim3(1), dim3(1), 0, st, 1u, sink);
    return hipGetLastError();
}

size_t batch_inverse_scratch(size_t n) {
    size_t tot = 0;
    while (n > BI_BASE) {
        n = (n + BI_WG - 1) / BI_WG;
        tot += 2 * n;
    }
    return tot;
}

hipError_t launch_batch_inverse(const Fr* in, Fr* out, size_t n, hipStream_t st, Fr* scratch, const Fr* inv_total) {
    if (!n) return hipSuccess;
    if (!scratch && n > BI_BASE) {
        // lanes for one wave per SIMD (256 CUs x 4 SIMDs x 64), 8 .. 256 elements each
        uint32_t chunk = 8;
        while (chunk < 256 && (size_t)chunk * 65536 < n) chunk *= 2;
        const size_t T = (n + chunk - 1) / chunk;
        hipLaunchKernelGGL(k_batch_inverse, dim3(nblocks(T, 256)), dim3(256), 0, st, in, out, n, T, chunk);
        return hipGetLastError();
    }
    if (n <= BI_BASE) {
        hipLaunchKernelGGL(k_bi_base, dim3(1), dim3(BI_THREADS), 0, st, in, out, n, inv_total ? *inv_total : fr_zero(),
                           inv_total ? 1 : 0);
        return hipGetLastError();
    }
    const size_t T = (n + BI_WG - 1) / BI_WG;  // workgroups of the up/down passes = products one level up
    Fr* prod = scratch;
    Fr* inv_prod = scratch + T;
    hipLaunchKernelGGL(k_bi_up, dim3((unsigned)T), dim3(BI_THREADS), 0, st, in, out, n, prod);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = launch_batch_inverse(prod, inv_prod, T, st, scratch + 2 * T, inv_total);  // same total product
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_bi_down, dim3((unsigned)T), dim3(BI_THREADS), 0, st, in, out, n, inv_prod);
    return hipGetLastError();
}

hipError_t launch_calib_mul(Fr* out, size_t nthreads, uint32_t iters, hipStream_t st) {
    hipLaunchKernelGGL(k_calib_mul, dim3(nblocks(nthreads, 256)), dim3(256), 0, st, out, iters);
    return hipGetLastError();
}

hipError_t launch_gather(const uint64_t* ptrs, Fr* out, size_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gather, dim3(nblocks(n, 256)), dim3(256), 0, st, ptrs, out, n);
    return hipGetLastError();
}

hipError_t launch_assemble_chunks(const Fr* stage, uint32_t logGq, size_t Sq, Fr* out, hipStream_t st) {
    const size_t n = Sq << logGq;
    hipLaunchKernelGGL(k_assemble_chunks, dim3(nblocks(n, 256)), dim3(256), 0, st, stage, logGq, Sq, out);
    return hipGetLastError();
}

}  // namespace lsp

LSP_BOUNDS_READER(k_field)
