// Coset LDE building blocks: transposes, LDS-tiled radix-2 NTT passes, power
// tables and the coset twist.  Together they implement
// Radix2DitParallel::coset_lde_batch ([EXT p3-dft], bin/src/config.rs:22).
//
// Layout: the batched NTT works on column-major scratch (one contiguous
// array of 2^logH elements per column and coset).  A pass fuses k radix-2
// stages in LDS on a tile of 2^k x G elements (G adjacent groups so every
// global access is >= 128 contiguous bytes); the whole transform is
// ceil(logH / 9) passes.  Fr is 32 bytes, so a 2048-element tile is 64 KiB
// of the CU's 160 KiB LDS (two workgroups per CU).
#include "k_common.hpp"
#include "kernels.hpp"

namespace lsp {

namespace {
constexpr unsigned TR = 64, TC = 8;  // transpose tile

__global__ __launch_bounds__(256) void k_transpose(const Fr* __restrict__ src, Fr* __restrict__ dst, size_t R,
                                                   size_t C, uint32_t logR, int bitrev_rows, uint32_t tilesR,
                                                   uint32_t tilesC) {
    __shared__ Fr tile[TR * TC];
    const uint64_t blk = blockIdx.x;
    const uint64_t per = (uint64_t)tilesR * tilesC;
    const uint64_t b = blk / per;
    const uint64_t rem = blk - b * per;
    const size_t r0 = (rem / tilesC) * TR, c0 = (rem % tilesC) * TC;
    const Fr* s = src + b * R * C;
    Fr* d = dst + b * R * C;
    for (unsigned e = threadIdx.x; e < TR * TC; e += blockDim.x) {
        unsigned r = e / TC, c = e % TC;
        size_t gr = r0 + r, gc = c0 + c;
        if (gr < R && gc < C) {
            size_t sr = bitrev_rows ? (size_t)brev_bits(gr, logR) : gr;
            tile[r * TC + c] = s[sr * C + gc];
        }
    }
    __syncthreads();
    for (unsigned e = threadIdx.x; e < TR * TC; e += blockDim.x) {
        unsigned c = e / TR, r = e % TR;
        size_t gr = r0 + r, gc = c0 + c;
        if (gr < R && gc < C) d[gc * R + gr] = tile[r * TC + c];
    }
}

template <bool DIF>
__global__ __launch_bounds__(256) void k_ntt_pass(Fr* __restrict__ data, const Fr* __restrict__ tw, uint32_t logH,
                                                  uint32_t s0, uint32_t k, uint32_t logL, uint32_t logG) {
    extern __shared__ Fr lds[];
    const uint32_t K = 1u << k, G = 1u << logG;
    const uint64_t H = 1ull << logH;
    const uint64_t tiles_per_arr = H >> (k + logG);
    const uint64_t wg = blockIdx.x;
    const uint64_t b = wg / tiles_per_arr, tile = wg - b * tiles_per_arr;
    Fr* arr = data + b * H;
    const uint64_t Lmask = (1ull << logL) - 1;
    const uint32_t n_el = K * G;
    const bool t_minor = logL < logG;
    for (uint32_t e = threadIdx.x; e < n_el; e += blockDim.x) {
        uint32_t t, g;
        if (t_minor) {
            t = e & (K - 1);
            g = e >> k;
        } else {
            t = e >> logG;
            g = e & (G - 1);
        }
        const uint64_t gid = tile * G + g;
        const uint64_t idx = ((gid >> logL) << (logL + k)) + ((uint64_t)t << logL) + (gid & Lmask);
        lds[t * G + g] = arr[idx];
    }
    __syncthreads();
    for (uint32_t j = 0; j < k; ++j) {
        const uint32_t s = s0 + j;
        const uint32_t logd = DIF ? (k - 1 - j) : j;
        for (uint32_t bf = threadIdx.x; bf < (n_el >> 1); bf += blockDim.x) {
            const uint32_t g = bf & (G - 1), p = bf >> logG;
            const uint32_t t0 = ((p >> logd) << (logd + 1)) | (p & ((1u << logd) - 1));
            const uint32_t t1 = t0 + (1u << logd);
            const uint64_t gid = tile * G + g;
            const uint64_t i0 = ((gid >> logL) << (logL + k)) + ((uint64_t)t0 << logL) + (gid & Lmask);
            uint64_t twi;
            if (DIF)
                twi = (i0 & ((H >> (s + 1)) - 1)) << s;
            else
                twi = (i0 & ((1ull << s) - 1)) << (logH - 1 - s);
            const Fr w = tw[twi];
            const Fr a = lds[t0 * G + g], c = lds[t1 * G + g];
            if (DIF) {
                lds[t0 * G + g] = fr_add(a, c);
                lds[t1 * G + g] = fr_mul(fr_sub(a, c), w);
            } else {
                const Fr cw = fr_mul(c, w);
                lds[t0 * G + g] = fr_add(a, cw);
                lds[t1 * G + g] = fr_sub(a, cw);
            }
        }
        __syncthreads();
    }
    for (uint32_t e = threadIdx.x; e < n_el; e += blockDim.x) {
        uint32_t t, g;
        if (t_minor) {
            t = e & (K - 1);
            g = e >> k;
        } else {
            t = e >> logG;
            g = e & (G - 1);
        }
        const uint64_t gid = tile * G + g;
        const uint64_t idx = ((gid >> logL) << (logL + k)) + ((uint64_t)t << logL) + (gid & Lmask);
        arr[idx] = lds[t * G + g];
    }
}

__global__ __launch_bounds__(256) void k_pow_tables(const Fr* __restrict__ bases, size_t nbases, uint32_t L1,
                                                    uint32_t L2, const Fr* __restrict__ scale,
                                                    Fr* __restrict__ tabs) {
    const size_t per = (1ull << L1) + (1ull << L2);
    const size_t i = gtid();
    if (i >= nbases * per) return;
    const size_t b = i / per, j = i - b * per;
    const Fr base = bases[b];
    if (j < (1ull << L1)) {
        tabs[i] = fr_pow_u64(base, j);
    } else {
        Fr v = fr_pow_u64(base, (uint64_t)(j - (1ull << L1)) << L1);
        if (scale) v = fr_mul(v, scale[b]);
        tabs[i] = v;
    }
}

__global__ __launch_bounds__(256) void k_powers(const Fr* __restrict__ tab, uint32_t L1, size_t n,
                                                Fr* __restrict__ out) {
    const size_t i = gtid();
    if (i < n) out[i] = pow2l(tab, L1, i);
}

__global__ __launch_bounds__(256) void k_twist_expand(const Fr* __restrict__ X, Fr* __restrict__ Y, size_t w,
                                                      uint32_t logh, uint32_t ncosets, const Fr* __restrict__ tabs,
                                                      uint32_t L1, uint32_t L2) {
    const size_t h = 1ull << logh;
    const size_t idx = gtid();
    if (idx >= (size_t)ncosets * w * h) return;
    const size_t arr = idx >> logh;  // k*w + c
    const size_t i = idx & (h - 1);
    const size_t c = arr % w;
    const Fr* tab = tabs + arr * ((1ull << L1) + (1ull << L2));
    Y[idx] = fr_mul(X[c * h + i], pow2l(tab, L1, i));
}
}  // namespace

hipError_t launch_transpose(const Fr* src, Fr* dst, size_t batch, size_t R, size_t C, bool bitrev_rows,
                            hipStream_t st) {
    uint32_t logR = 0;
    while ((1ull << logR) < R) ++logR;
    const uint32_t tR = (uint32_t)((R + TR - 1) / TR), tC = (uint32_t)((C + TC - 1) / TC);
    const size_t nb = batch * tR * tC;
    hipLaunchKernelGGL(k_transpose, dim3((unsigned)nb), dim3(256), 0, st, src, dst, R, C, logR,
                       bitrev_rows ? 1 : 0, tR, tC);
    return hipGetLastError();
}

hipError_t launch_ntt(Fr* data, size_t batch, uint32_t logH, const Fr* tw, bool dif, hipStream_t st) {
    if (logH == 0) return hipSuccess;
    // plan: passes of <= 9 stages (G = 4) or one pass of logH <= 11 stages (G = 1)
    uint32_t ks[8], np = 0;
    if (logH <= 11) {
        ks[np++] = logH;
    } else {
        uint32_t P = (logH + 8) / 9;
        for (uint32_t p = 0; p < P; ++p) ks[np++] = logH / P + (p < logH % P ? 1 : 0);
    }
    uint32_t s0 = 0;
    for (uint32_t p = 0; p < np; ++p) {
        const uint32_t k = ks[p];
        const uint32_t logG = (logH - k) < 2 ? (logH - k) : 2;
        const uint32_t logL = dif ? (logH - s0 - k) : s0;
        const uint64_t tiles = (batch << logH) >> (k + logG);
        const size_t lds = (size_t(1) << (k + logG)) * sizeof(Fr);
        if (dif)
            hipLaunchKernelGGL(k_ntt_pass<true>, dim3((unsigned)tiles), dim3(256), lds, st, data, tw, logH, s0, k,
                               logL, logG);
        else
            hipLaunchKernelGGL(k_ntt_pass<false>, dim3((unsigned)tiles), dim3(256), lds, st, data, tw, logH, s0,
                               k, logL, logG);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        s0 += k;
    }
    return hipSuccess;
}

hipError_t launch_pow_tables(const Fr* bases, size_t nbases, uint32_t L1, uint32_t L2, const Fr* scale, Fr* tabs,
                             hipStream_t st) {
    const size_t n = nbases * ((1ull << L1) + (1ull << L2));
    hipLaunchKernelGGL(k_pow_tables, dim3(nblocks(n, 256)), dim3(256), 0, st, bases, nbases, L1, L2, scale, tabs);
    return hipGetLastError();
}

hipError_t launch_powers(const Fr* tab, uint32_t L1, size_t n, Fr* out, hipStream_t st) {
    hipLaunchKernelGGL(k_powers, dim3(nblocks(n, 256)), dim3(256), 0, st, tab, L1, n, out);
    return hipGetLastError();
}

hipError_t launch_twist_expand(const Fr* X, Fr* Y, size_t w, uint32_t logh, uint32_t ncosets, const Fr* tabs,
                               uint32_t L1, uint32_t L2, hipStream_t st) {
    const size_t n = (size_t)ncosets * w << logh;
    hipLaunchKernelGGL(k_twist_expand, dim3(nblocks(n, 256)), dim3(256), 0, st, X, Y, w, logh, ncosets, tabs, L1,
                       L2);
    return hipGetLastError();
}

}  // namespace lsp
