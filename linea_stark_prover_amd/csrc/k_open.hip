// TwoAdicFriPcs::open building blocks ([EXT p3-fri]): inverse denominators
// 1/(z - GEN w_N^bitrev(i)), barycentric opened values (interpolate_coset),
// the "reduce rows" accumulation, and the FRI fold
// (TwoAdicFriGenericConfig::fold_matrix).
#include "fr29.hpp"
#include "k_common.hpp"
#include "kernels.hpp"

namespace lsp {

namespace {
__global__ __launch_bounds__(256) void k_open_denoms(Fr z, Fr gen, const Fr* __restrict__ tabN, uint32_t L1,
                                                     uint32_t logN, size_t n, uint64_t row0,
                                                     Fr* __restrict__ den) {
    const size_t i = gtid();
    if (i >= n) return;
    den[i] = fr_sub(z, fr_mul(gen, pow2l(tabN, L1, brev_bits(row0 + i, logN))));
}

// 1/(z w_h - x) = w_h^-1 / (z - x w_h^-1), and x w_h^-1 is the domain point
// `step` = N/h positions earlier in natural order: the inverse denominators of
// zeta_next are a permuted, scaled copy of zeta's.  Row j = bitrev(bitrev(i) - step)
// keeps the low log_blowup bits of the natural index, i.e. the same shard.
__global__ __launch_bounds__(256) void k_shift_inverse(const Fr* __restrict__ inv_z, Fr* __restrict__ out, Fr c,
                                                       uint32_t logN, uint64_t step, uint64_t row0, size_t n) {
    const size_t i = gtid();
    if (i >= n) return;
    const uint64_t nat = brev_bits(row0 + i, logN);
    const uint64_t j = brev_bits((nat - step) & ((1ull << logN) - 1), logN) - row0;
    out[i] = fr_mul(c, inv_z[j]);
}

constexpr uint32_t INTERP_ROWS = 1024;  // rows per block

// partial[b*w + c] = sum over the block's rows i of M[i][c] * x_i * inv_den[i]
// The row factors x_i inv_den[i] go into LDS once per block in the 29-bit form,
// so every M[i][c] (ark form) times its factor is the 29-bit product (ark form
// out, as in k_reduce_rows), accumulated lazily and reduced every RR_CHUNK
// products through the LDS table; the column sums leave canonical.
constexpr uint32_t RR_CHUNK = 3;  // 3 normalised products + a value < 2r: limbs < 2^31, < 26.2 r (f29_reduce_qt)
__global__ __launch_bounds__(256) void k_interp_partial(const Fr* __restrict__ M, uint32_t w, size_t h,
                                                        const Fr* __restrict__ inv_den, Fr gen,
                                                        const Fr* __restrict__ tabN, uint32_t L1, uint32_t logN,
                                                        Fr* __restrict__ partial, uint64_t row0) {
    __shared__ Fr red[256];
    __shared__ F29 sc[INTERP_ROWS];
    __shared__ uint4 qt[3 * F29_QTAB_N];
    f29_qtab_init(qt);
    const size_t r0 = (size_t)blockIdx.x * INTERP_ROWS;
    const uint32_t nr = (uint32_t)min((size_t)INTERP_ROWS, h - r0);
    for (uint32_t e = threadIdx.x; e < nr; e += blockDim.x)
        sc[e] = f29_from_fr(fr_mul(fr_mul(gen, pow2l(tabN, L1, brev_bits(row0 + r0 + e, logN))), inv_den[r0 + e]));
    __syncthreads();
    // the threads as R row lanes x W adjacent columns (W = min(w, 256)): one step
    // reads W adjacent elements of R consecutive rows, a contiguous run of the
    // row-major matrix; one LDS sum per column chunk instead of a tree per column
    const uint32_t W = min(w, 256u), R = 256u / W;
    const uint32_t cc = threadIdx.x % W, rr = threadIdx.x / W;
    for (uint32_t c0 = 0; c0 < w; c0 += W) {
        const uint32_t c = c0 + cc;
        Fr acc = fr_zero();
        if (rr < R && c < w) {
            F29 s = f29_zero();
            uint32_t k = 0;
            for (uint32_t r = rr; r < nr; r += R) {
                s = f29_lazy2(s, f29_mul(f29_repack_in(M[(r0 + r) * w + c]), sc[r]));  // < 8.06 r each
                if (++k == RR_CHUNK) {
                    s = f29_reduce_qt(s, qt);  // < 2 r
                    k = 0;
                }
            }
            acc = fr_reduce_once(f29_repack_out(f29_reduce_qt(s, qt)));
        }
        red[threadIdx.x] = acc;
        __syncthreads();
        if (threadIdx.x < W && c0 + threadIdx.x < w) {
            Fr sum = red[threadIdx.x];
            for (uint32_t k = 1; k < R; ++k) sum = fr_add(sum, red[threadIdx.x + k * W]);
            partial[(size_t)blockIdx.x * w + c0 + threadIdx.x] = sum;
        }
        __syncthreads();
    }
}

static_assert(sizeof(F29) == 36, "reduce_rows_scratch (kernels.hpp) assumes 36-byte F29");

// one workgroup per column: strided partial sums, then a tree in LDS
__global__ __launch_bounds__(256) void k_sum_partials(const Fr* __restrict__ partial, uint32_t nb, uint32_t w,
                                                      Fr* __restrict__ out) {
    __shared__ Fr red[256];
    const uint32_t c = blockIdx.x;
    Fr acc = fr_zero();
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) acc = fr_add(acc, partial[(size_t)b * w + c]);
    red[threadIdx.x] = acc;
    __syncthreads();
    for (uint32_t s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] = fr_add(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) out[c] = red[0];
}

// One row of the FRI input: (ry_z - rr) / (z - x) + apw[w] (ry_zn - rr) / (zn - x)
// + sum_j apw[2w+j] (ryq_j - qrow_j) / (z - x), rr = sum_k apw[k] row[k].
// On the 29-bit-limb product (fr29.hpp): an ark-form element X = x 2^256 times
// the 29-bit form W = w 2^261 gives X W 2^-261 = the ark form of x w, so the
// constants (alpha powers) are converted once per workgroup into LDS and every
// per-row factor (the inverse denominators) once per row; sums stay lazily
// reduced (at most 3 products per limb-wise sum, then the LDS-table
// reduction).  The result is canonical.
// the per-call constants of k_reduce_rows in their kernel form: apw[0..w] and
// apw[2w..2w+q) in the 29-bit form, then ryq[0..q) as limbs (ark form)
__device__ __forceinline__ F29 rr_const(const ReduceArgs& a, uint32_t k) {
    if (k <= a.w) return f29_from_fr(a.apw[k]);
    if (k < a.w + 1 + a.q) return f29_from_fr(a.apw[2 * a.w + (k - a.w - 1)]);
    return f29_repack_in(a.ryq[k - a.w - 1 - a.q]);
}

// wide matrices (GLB, the constants beyond the LDS): converted once into global memory
__global__ __launch_bounds__(256) void k_reduce_consts(ReduceArgs a) {
    const size_t k = gtid();
    if (k < a.w + 1 + 2 * (size_t)a.q) a.consts29[k] = rr_const(a, (uint32_t)k);
}

// GLB: the constants come from a.consts29 (k_reduce_consts) instead of the
// workgroup's LDS -- for w + 2q beyond the LDS (about 4,400 columns)
template <bool GLB>
__global__ __launch_bounds__(256) void k_reduce_rows(ReduceArgs a) {
    extern __shared__ uint4 rr_lds[];
    uint4* qt = rr_lds;                                               // 3 * F29_QTAB_N
    const F29* apw29;  // apw[0..w], apw[2w..2w+q): 29-bit form
    f29_qtab_init(qt);
    if constexpr (GLB) {
        apw29 = a.consts29;
    } else {
        F29* c = reinterpret_cast<F29*>(rr_lds + 3 * F29_QTAB_N);
        for (uint32_t k = threadIdx.x; k < a.w + 1 + 2 * a.q; k += blockDim.x) c[k] = rr_const(a, k);
        apw29 = c;
    }
    const F29* ryq_l = apw29 + a.w + 1 + a.q;  // ryq[j] as limbs (ark form)
    __syncthreads();
    const size_t i = gtid();
    if (i >= a.n) return;
    // the constants' LDS copy: the launch sized it for w + 1 + 2q entries after the table
    if (!LSP_BOUNDS(GLB || 3 * F29_QTAB_N * sizeof(uint4) + (a.w + 1 + 2 * (size_t)a.q) * sizeof(F29) <= a.lds_max))
        return;
    const Fr* row = a.lde + i * a.w;
    const Fr* qrow = a.qlde + i * a.q;
    // Software-pipelined loads: the next chunk of the row (then of the quotient
    // row) is requested before the current chunk's products, so a wave waits
    // for HBM about once per row instead of once per element (the loads used to
    // sit right before their products, ~1/3 of the kernel's cycles stalled).
    constexpr uint32_t RC = RR_CHUNK;
    auto load = [&](const Fr* p, uint32_t n, uint32_t k, Fr* dst) {
#pragma unroll
        for (uint32_t j = 0; j < RC; ++j)
            if (k + j < n) dst[j] = p[k + j];
    };
    const Fr zi = a.inv_z[i], zni = a.inv_zn[i];
    Fr cur[RC], nxt[RC];
    if (a.w)
        load(row, a.w, 0, cur);
    else
        load(qrow, a.q, 0, cur);
    F29 rr = f29_zero();
    for (uint32_t k = 0; k < a.w; k += RC) {
        if (k + RC < a.w)
            load(row, a.w, k + RC, nxt);
        else
            load(qrow, a.q, 0, nxt);  // the quotient row's first chunk
        F29 s = rr;
#pragma unroll
        for (uint32_t j = 0; j < RC; ++j)
            if (k + j < a.w) s = f29_lazy2(s, f29_mul(f29_repack_in(cur[j]), apw29[k + j]));  // < 8.06 r each
        rr = f29_reduce_qt(s, qt);  // < 2 r
#pragma unroll
        for (uint32_t j = 0; j < RC; ++j) cur[j] = nxt[j];
    }
    const F29 iz = f29_from_fr(zi), izn = f29_from_fr(zni);  // 29-bit form, < 2 r
    const F29 t1 = f29_mul(f29_sub16(f29_repack_in(a.ry_z), rr), iz);          // < 17 r in, < 8.1 r out
    const F29 t2 = f29_mul(f29_mul(f29_sub16(f29_repack_in(a.ry_zn), rr), izn), apw29[a.w]);
    F29 qacc = f29_zero();
    for (uint32_t k = 0; k < a.q; k += RC) {
        if (k + RC < a.q) load(qrow, a.q, k + RC, nxt);
        F29 s = qacc;
#pragma unroll
        for (uint32_t j = 0; j < RC; ++j)
            if (k + j < a.q)
                s = f29_lazy2(s, f29_mul(f29_sub16(ryq_l[k + j], f29_repack_in(cur[j])), apw29[a.w + 1 + k + j]));
        qacc = f29_reduce_qt(s, qt);
#pragma unroll
        for (uint32_t j = 0; j < RC; ++j) cur[j] = nxt[j];
    }
    const F29 t3 = f29_mul(qacc, iz);
    a.out[i] = fr_reduce_once(f29_repack_out(f29_reduce_qt(f29_lazy3(t1, t2, t3), qt)));  // < 24.3 r in
}

// coef[0..npts) = alpha offsets, coef[npts..2 npts) = offset * reduced ys; apw = alpha^c, c < w
__global__ __launch_bounds__(256) void k_reduce_matrix(const Fr* __restrict__ M, size_t n, uint32_t w,
                                                       const Fr* __restrict__ apw, uint32_t npts,
                                                       const Fr* __restrict__ inv, const Fr* __restrict__ off,
                                                       const Fr* __restrict__ offys, Fr* __restrict__ ro) {
    const size_t i = gtid();
    if (i >= n) return;
    const Fr* row = M + i * w;
    Fr rr = fr_zero();
    for (uint32_t c = 0; c < w; ++c) rr = fr_add(rr, fr_mul(apw[c], row[c]));
    Fr acc = ro[i];
    for (uint32_t p = 0; p < npts; ++p)
        acc = fr_add(acc, fr_mul(fr_sub(offys[p], fr_mul(off[p], rr)), inv[(size_t)p * n + i]));
    ro[i] = acc;
}

__global__ __launch_bounds__(256) void k_fri_fold(const Fr* __restrict__ v, size_t m, Fr half, Fr half_beta,
                                                  const Fr* __restrict__ tab, uint32_t L1, uint32_t logm,
                                                  uint64_t i0, Fr* __restrict__ out) {
    const size_t i = gtid();
    if (i >= m) return;
    const Fr p = fr_mul(half_beta, pow2l(tab, L1, brev_bits(i0 + i, logm)));
    out[i] = fr_add(fr_mul(fr_add(half, p), v[2 * i]), fr_mul(fr_sub(half, p), v[2 * i + 1]));
}
}  // namespace

hipError_t launch_open_denoms(Fr z, Fr gen, const Fr* tabN, uint32_t L1, uint32_t logN, size_t n, Fr* den,
                              hipStream_t st, uint64_t row0) {
    hipLaunchKernelGGL(k_open_denoms, dim3(nblocks(n, 256)), dim3(256), 0, st, z, gen, tabN, L1, logN, n, row0,
                       den);
    return hipGetLastError();
}

hipError_t launch_shift_inverse(const Fr* inv_z, Fr* out, Fr c, uint32_t logN, uint64_t step, uint64_t row0, size_t n,
                                hipStream_t st) {
    hipLaunchKernelGGL(k_shift_inverse, dim3(nblocks(n, 256)), dim3(256), 0, st, inv_z, out, c, logN, step, row0, n);
    return hipGetLastError();
}

hipError_t launch_interp_partial(const Fr* M, uint32_t w, size_t h, const Fr* inv_den, Fr gen, const Fr* tabN,
                                 uint32_t L1, uint32_t logN, Fr* partial, uint32_t* nb, hipStream_t st, uint64_t row0) {
    *nb = (uint32_t)((h + INTERP_ROWS - 1) / INTERP_ROWS);
    hipLaunchKernelGGL(k_interp_partial, dim3(*nb), dim3(256), 0, st, M, w, h, inv_den, gen, tabN, L1, logN,
                       partial, row0);
    return hipGetLastError();
}

hipError_t launch_sum_partials(const Fr* partial, uint32_t nb, uint32_t w, Fr* out, hipStream_t st) {
    hipLaunchKernelGGL(k_sum_partials, dim3(w), dim3(256), 0, st, partial, nb, w, out);
    return hipGetLastError();
}

hipError_t launch_reduce_rows(const ReduceArgs& a, hipStream_t st) {
    const size_t qtab = 3 * F29_QTAB_N * sizeof(uint4);
    const size_t nconst = a.w + 1 + 2 * (size_t)a.q;
    const size_t lds = qtab + nconst * sizeof(F29);
    if (lds <= a.lds_max) {
        hipLaunchKernelGGL(k_reduce_rows<false>, dim3(nblocks(a.n, 256)), dim3(256), lds, st, a);
        return hipGetLastError();
    }
    if (!a.consts29) return hipErrorInvalidValue;  // the caller must pass the global scratch (reduce_rows_scratch)
    hipLaunchKernelGGL(k_reduce_consts, dim3(nblocks(nconst, 256)), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_reduce_rows<true>, dim3(nblocks(a.n, 256)), dim3(256), qtab, st, a);
    return hipGetLastError();
}

hipError_t launch_reduce_matrix(const Fr* M, size_t n, uint32_t w, const Fr* apw, uint32_t npts, const Fr* inv,
                                const Fr* off, const Fr* offys, Fr* ro, hipStream_t st) {
    hipLaunchKernelGGL(k_reduce_matrix, dim3(nblocks(n, 256)), dim3(256), 0, st, M, n, w, apw, npts, inv, off, offys,
                       ro);
    return hipGetLastError();
}

hipError_t launch_fri_fold(const Fr* v, size_t m, Fr half, Fr half_beta, const Fr* tab, uint32_t L1, Fr* out,
                           hipStream_t st, uint64_t i0, int logm) {
    uint32_t lg = 0;
    if (logm >= 0)
        lg = (uint32_t)logm;
    else
        while ((1ull << lg) < m) ++lg;
    hipLaunchKernelGGL(k_fri_fold, dim3(nblocks(m, 256)), dim3(256), 0, st, v, m, half, half_beta, tab, L1, lg, i0,
                       out);
    return hipGetLastError();
}

}  // namespace lsp

LSP_BOUNDS_READER(k_open)
