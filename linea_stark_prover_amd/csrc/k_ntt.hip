// Coset LDE on row-major matrices: Radix2DitParallel::coset_lde_batch
// ([EXT p3-dft], bin/src/config.rs:22) as TwoAdicFriPcs::commit uses it.
//
// Data never leaves the row-major layout the prover hashes:
//   inverse   DIT passes over X (h x w): the first pass gathers the caller's
//             rows in bit-reversed order, so X ends as h * coefficients in
//             natural order;
//   forward   for every coset k, DIF passes over block k of the output
//             (rows k*h .. (k+1)*h - 1): the first pass multiplies coefficient
//             i of column c by s_{k,c}^i / h on load (the coset twist), the
//             last pass leaves the block in bit-reversed order -- exactly
//             rows k*h + u = p_c(s_{k,c} w_h^bitrev(u)), the bit-reversed LDE.
// A pass fuses k <= 8 radix-2 stages in LDS on a tile of 2^k positions x G
// adjacent groups x CW adjacent columns (CW*G = 8: every global access is a
// 256-byte run of a row, or of adjacent rows).  Fr is 32 bytes; a tile is at
// most 2048 elements = 64 KiB of the CU's 160 KiB LDS.  Butterflies whose
// twiddle is 1 (DIT stage 0, DIF last stage) skip the product.
#include "k_common.hpp"
#include "kernels.hpp"

namespace lsp {

namespace {
enum PassMode : int { PASS_INPLACE = 0, PASS_INV_FIRST = 1, PASS_FWD_FIRST = 2 };

struct NttPass {
    const Fr* src;      // PASS_INV_FIRST: caller rows; PASS_FWD_FIRST: X (coefficients)
    Fr* dst;            // the arrays being transformed (h rows each, batch of `narr` arrays, row-major w)
    const Fr* tw;       // w_H^x (or inverse), x < H/2
    const Fr* twist;    // PASS_FWD_FIRST: two-level tables per (coset[, column])
    uint32_t L1, L2;    // twist table split
    uint32_t twist_per_col;  // 1: table index k*w + c, 0: table index k
    uint32_t logH, s0, k, logL, logG, CW, w;
    uint64_t narr;      // arrays (cosets) in dst
};

template <bool DIF, int MODE>
__global__ __launch_bounds__(256) void k_ntt_rm(NttPass p) {
    extern __shared__ Fr lds[];
    const uint32_t K = 1u << p.k, G = 1u << p.logG, CW = p.CW;
    const uint64_t H = 1ull << p.logH;
    const uint32_t nchunk = (p.w + CW - 1) / CW;
    const uint64_t tiles_per_arr = (H >> (p.k + p.logG)) * nchunk;
    const uint64_t wg = blockIdx.x;
    const uint64_t arr = wg / tiles_per_arr;
    const uint64_t rem = wg - arr * tiles_per_arr;
    const uint64_t tile = rem / nchunk;
    const uint32_t c0 = (uint32_t)(rem - tile * nchunk) * CW;
    const uint32_t cw = min(CW, p.w - c0);
    const uint64_t Lmask = (1ull << p.logL) - 1;
    const uint32_t n_el = K * G * CW;
    const bool t_minor = p.logL < p.logG;
    Fr* base = p.dst + arr * H * p.w;
    // ---- load (optionally gathering / twisting)
    for (uint32_t e = threadIdx.x; e < n_el; e += blockDim.x) {
        const uint32_t c = e % CW;
        const uint32_t tg = e / CW;
        uint32_t t, g;
        if (t_minor) {
            t = tg & (K - 1);
            g = tg >> p.k;
        } else {
            t = tg >> p.logG;
            g = tg & (G - 1);
        }
        if (c >= cw) continue;
        const uint64_t gid = tile * G + g;
        const uint64_t row = ((gid >> p.logL) << (p.logL + p.k)) + ((uint64_t)t << p.logL) + (gid & Lmask);
        Fr v;
        if (MODE == PASS_INV_FIRST) {
            v = p.src[brev_bits(row, p.logH) * p.w + c0 + c];
        } else if (MODE == PASS_FWD_FIRST) {
            const uint64_t ti = p.twist_per_col ? (arr * p.w + c0 + c) : arr;
            const Fr* tab = p.twist + ti * ((1ull << p.L1) + (1ull << p.L2));
            v = fr_mul(p.src[row * p.w + c0 + c], pow2l(tab, p.L1, row));
        } else {
            v = base[row * p.w + c0 + c];
        }
        lds[(t * G + g) * CW + c] = v;
    }
    __syncthreads();
    // ---- k radix-2 stages
    const uint32_t nbf = n_el >> 1;
    for (uint32_t j = 0; j < p.k; ++j) {
        const uint32_t s = p.s0 + j;
        const uint32_t logd = DIF ? (p.k - 1 - j) : j;
        const bool trivial = DIF ? (s == p.logH - 1) : (s == 0);
        for (uint32_t bf = threadIdx.x; bf < nbf; bf += blockDim.x) {
            const uint32_t c = bf % CW;
            const uint32_t pg = bf / CW;
            const uint32_t g = pg & (G - 1), pp = pg >> p.logG;
            const uint32_t t0 = ((pp >> logd) << (logd + 1)) | (pp & ((1u << logd) - 1));
            const uint32_t t1 = t0 + (1u << logd);
            const uint32_t a0 = (t0 * G + g) * CW + c, a1 = (t1 * G + g) * CW + c;
            const Fr a = lds[a0], b = lds[a1];
            if (trivial) {
                lds[a0] = fr_add(a, b);
                lds[a1] = fr_sub(a, b);
                continue;
            }
            const uint64_t gid = tile * G + g;
            const uint64_t i0 = ((gid >> p.logL) << (p.logL + p.k)) + ((uint64_t)t0 << p.logL) + (gid & Lmask);
            uint64_t twi;
            if (DIF)
                twi = (i0 & ((H >> (s + 1)) - 1)) << s;
            else
                twi = (i0 & ((1ull << s) - 1)) << (p.logH - 1 - s);
            const Fr wv = p.tw[twi];
            if (DIF) {
                lds[a0] = fr_add(a, b);
                lds[a1] = fr_mul(fr_sub(a, b), wv);
            } else {
                const Fr bw = fr_mul(b, wv);
                lds[a0] = fr_add(a, bw);
                lds[a1] = fr_sub(a, bw);
            }
        }
        __syncthreads();
    }
    // ---- store
    for (uint32_t e = threadIdx.x; e < n_el; e += blockDim.x) {
        const uint32_t c = e % CW;
        const uint32_t tg = e / CW;
        uint32_t t, g;
        if (t_minor) {
            t = tg & (K - 1);
            g = tg >> p.k;
        } else {
            t = tg >> p.logG;
            g = tg & (G - 1);
        }
        if (c >= cw) continue;
        const uint64_t gid = tile * G + g;
        const uint64_t row = ((gid >> p.logL) << (p.logL + p.k)) + ((uint64_t)t << p.logL) + (gid & Lmask);
        base[row * p.w + c0 + c] = lds[(t * G + g) * CW + c];
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

void plan_passes(uint32_t logH, uint32_t kmax, uint32_t* ks, uint32_t& np) {
    np = 0;
    if (logH <= kmax) {
        ks[np++] = logH;
        return;
    }
    const uint32_t P = (logH + kmax - 1) / kmax;
    for (uint32_t q = 0; q < P; ++q) ks[np++] = logH / P + (q < logH % P ? 1 : 0);
}
}  // namespace

hipError_t launch_lde(const Fr* in, Fr* X, Fr* out, size_t w, uint32_t logh, uint32_t ncosets, const Fr* tw_inv,
                      const Fr* tw_fwd, const Fr* twist, uint32_t L1, uint32_t L2, int twist_per_col,
                      hipStream_t st) {
    if (w == 0) return hipSuccess;
    const uint32_t CW = (uint32_t)(w < 8 ? w : 8);
    const uint32_t Gmax = 8 / CW;
    uint32_t logGmax = 0;
    while ((2u << logGmax) <= Gmax) ++logGmax;
    const uint32_t nchunk = (uint32_t)((w + CW - 1) / CW);
    // k <= log2(2048 / (CW * G)) with CW * G <= 8
    const uint32_t kmax = 8;
    uint32_t ks[16], np;
    auto run = [&](bool dif, uint32_t narr, const Fr* src, Fr* dst, const Fr* tw, int first_mode) -> hipError_t {
        plan_passes(logh, kmax, ks, np);
        uint32_t s0 = 0;
        for (uint32_t q = 0; q < np; ++q) {
            const uint32_t k = ks[q];
            const uint32_t logG = (logh - k) < logGmax ? (logh - k) : logGmax;
            NttPass p;
            p.src = src;
            p.dst = dst;
            p.tw = tw;
            p.twist = twist;
            p.L1 = L1;
            p.L2 = L2;
            p.twist_per_col = (uint32_t)twist_per_col;
            p.logH = logh;
            p.s0 = s0;
            p.k = k;
            p.logL = dif ? (logh - s0 - k) : s0;
            p.logG = logG;
            p.CW = CW;
            p.w = (uint32_t)w;
            p.narr = narr;
            const uint64_t tiles = (uint64_t)narr * ((1ull << logh) >> (k + logG)) * nchunk;
            const size_t lds = (size_t(1) << (k + logG)) * CW * sizeof(Fr);
            const int mode = q == 0 ? first_mode : PASS_INPLACE;
            if (dif) {
                if (mode == PASS_FWD_FIRST)
                    hipLaunchKernelGGL((k_ntt_rm<true, PASS_FWD_FIRST>), dim3((unsigned)tiles), dim3(256), lds, st, p);
                else
                    hipLaunchKernelGGL((k_ntt_rm<true, PASS_INPLACE>), dim3((unsigned)tiles), dim3(256), lds, st, p);
            } else {
                if (mode == PASS_INV_FIRST)
                    hipLaunchKernelGGL((k_ntt_rm<false, PASS_INV_FIRST>), dim3((unsigned)tiles), dim3(256), lds, st, p);
                else
                    hipLaunchKernelGGL((k_ntt_rm<false, PASS_INPLACE>), dim3((unsigned)tiles), dim3(256), lds, st, p);
            }
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
            s0 += k;
        }
        return hipSuccess;
    };
    if (logh == 0) {
        // h = 1: the coefficient is the value; every coset row equals it
        hipError_t e = hipMemcpyAsync(X, in, w * sizeof(Fr), hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return e;
        for (uint32_t k = 0; k < ncosets; ++k) {
            e = hipMemcpyAsync(out + (size_t)k * w, X, w * sizeof(Fr), hipMemcpyDeviceToDevice, st);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    hipError_t e = run(false, 1, in, X, tw_inv, PASS_INV_FIRST);
    if (e != hipSuccess) return e;
    return run(true, ncosets, X, out, tw_fwd, PASS_FWD_FIRST);
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

}  // namespace lsp
