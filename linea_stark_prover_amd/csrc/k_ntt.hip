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
// A pass fuses k <= 7 radix-2 stages in LDS on a tile of 2^k positions x G
// adjacent groups x CW adjacent columns (CW*G = 8: every global access is a
// 256-byte run of a row, or of adjacent rows).  Butterflies whose twiddle is 1
// (DIT stage 0, DIF last stage) skip the product.
//
// Arithmetic: the 29-bit-limb Montgomery product (fr29.hpp, R' = 2^261) on
// ark-form elements.  An element X = x 2^256 is repacked bit for bit into 29-bit
// limbs; twiddles and twist factors are stored in the 29-bit Montgomery form
// W = w 2^261 (fr_to_f29form); the product X W 2^-261 = x w 2^256 is the ark
// form of x w -- no conversion product anywhere.  Inside a pass the tile lives
// in LDS in limb form (36 B per element), lazily reduced: every stored value is
// normalised and < 8.3 r (sums reduced to < 2r, products < 8.06 r); a - b is
// formed carry-free as a + 16r - b (f29_sub16).  Between passes the arrays hold
// ark words reduced to < 2r; only the last forward pass writes canonical words.
#include "fr29.hpp"
#include "k_common.hpp"
#include "kernels.hpp"

namespace lsp {

namespace {
enum PassMode : int { PASS_INPLACE = 0, PASS_INV_FIRST = 1, PASS_FWD_FIRST = 2 };

struct NttPass {
    const Fr* src;      // PASS_INV_FIRST: caller rows; PASS_FWD_FIRST: X (coefficients)
    Fr* dst;            // the arrays being transformed (h rows each, batch of `narr` arrays, row-major w)
    const uint4* tw;    // w_H^x (or inverse), x < H/2: 29-bit limbs, 3 x uint4 per element
    const Fr* twist;    // PASS_FWD_FIRST: two-level tables per (coset[, column])
    uint32_t L1, L2;    // twist table split
    uint32_t twist_per_col;  // 1: table index k*w + c, 0: table index k
    uint32_t logH, s0, k, logL, logG, w;
    uint32_t nchunk;    // column chunks of 2^LOGCW per row
    uint32_t canon;     // 1: write canonical words (the transform's last pass)
    uint64_t narr;      // arrays (cosets) in dst
};

// x^i from a two-level table of 29-bit-form factors: the product of two
// 29-bit-form values is the 29-bit form of the product
__device__ __forceinline__ F29 pow2l29(const Fr* tab, uint32_t L1, uint64_t i) {
    const F29 lo = f29_repack_in(tab[i & ((1ull << L1) - 1)]);
    const F29 hi = f29_repack_in(tab[(1ull << L1) + (i >> L1)]);
    return f29_mul(lo, hi);
}

// 9 limbs from a 48-byte padded slot (two 16-byte loads and one 4-byte load)
__device__ __forceinline__ F29 f29_load48(const uint4* __restrict__ q) {
    const uint4 a = q[0], b = q[1];
    F29 o;
    o.l[0] = a.x; o.l[1] = a.y; o.l[2] = a.z; o.l[3] = a.w;
    o.l[4] = b.x; o.l[5] = b.y; o.l[6] = b.z; o.l[7] = b.w;
    o.l[8] = reinterpret_cast<const uint32_t*>(q + 2)[0];
    return o;
}

__device__ __forceinline__ Fr f29_store(const F29& v, bool canon) {
    const Fr o = f29_repack_out(f29_reduce(v));  // < 2r
    return canon ? fr_reduce_once(o) : o;
}

// One tile: 2^k positions x 2^logG groups x 2^LOGCW columns (power-of-two
// chunk, so every index below is shifts and masks; rows are 32-bit within
// an array, H <= 2^31).  The first forward pass (PASS_FWD_FIRST) runs one
// workgroup per tile of the coefficients for ALL cosets: the tile is read
// from X once into registers (<= 4 elements per thread) and twisted, transformed
// and stored once per coset, so X is not re-read for every coset.
constexpr uint32_t NTT_THREADS = 256;
constexpr uint32_t NTT_MAX_EL = 1024;  // 2^k x G x CW <= 2^7 x 8

template <bool DIF, int MODE, int LOGCW>
__global__ __launch_bounds__(NTT_THREADS) void k_ntt_rm(NttPass p) {
    extern __shared__ F29 lds[];
    constexpr uint32_t CW = 1u << LOGCW;
    constexpr bool FWD_FIRST = MODE == PASS_FWD_FIRST;
    const uint32_t K = 1u << p.k, logG = p.logG, G = 1u << logG;
    const uint32_t logL = p.logL, Lmask = (1u << logL) - 1, rowshift = logL + p.k;
    const uint64_t H = 1ull << p.logH;
    const uint32_t tiles_per_arr = (uint32_t)(H >> (p.k + logG)) * p.nchunk;
    const uint32_t wg = blockIdx.x;
    const uint32_t arr0 = FWD_FIRST ? 0u : wg / tiles_per_arr;
    const uint32_t arr_end = FWD_FIRST ? (uint32_t)p.narr : arr0 + 1;
    const uint32_t rem = wg - arr0 * tiles_per_arr;
    const uint32_t tile = rem / p.nchunk;
    const uint32_t c0 = (rem - tile * p.nchunk) << LOGCW;
    const uint32_t cw = min(CW, p.w - c0);
    const uint32_t n_el = (K << logG) << LOGCW;
    const bool t_minor = logL < logG;
    const uint32_t gid0 = tile << logG;
    auto row_of = [&](uint32_t t, uint32_t g) {
        const uint32_t gid = gid0 + g;
        return ((gid >> logL) << rowshift) + (t << logL) + (gid & Lmask);
    };
    auto split = [&](uint32_t e, uint32_t& t, uint32_t& g, uint32_t& c) {
        c = e & (CW - 1);
        const uint32_t tg = e >> LOGCW;
        if (t_minor) {
            t = tg & (K - 1);
            g = tg >> p.k;
        } else {
            t = tg >> logG;
            g = tg & (G - 1);
        }
    };
    // ---- first forward pass: this thread's coefficients of the tile, read once
    constexpr uint32_t NREG = FWD_FIRST ? NTT_MAX_EL / NTT_THREADS : 1;
    F29 xr[NREG];
    if (FWD_FIRST) {
#pragma unroll
        for (uint32_t j = 0; j < NREG; ++j) {
            const uint32_t e = threadIdx.x + j * NTT_THREADS;
            uint32_t t, g, c;
            split(e, t, g, c);
            if (e < n_el && c < cw) xr[j] = f29_repack_in(p.src[(size_t)row_of(t, g) * p.w + c0 + c]);
        }
    }
    F29* fac = lds + n_el;  // K * G extra entries (launcher sizes the LDS for it)
    const bool row_twist = FWD_FIRST && !p.twist_per_col;
    for (uint32_t arr = arr0; arr < arr_end; ++arr) {
        Fr* base = p.dst + (size_t)arr * H * p.w;
        if (FWD_FIRST && arr > arr0) __syncthreads();  // the previous coset's stores have read the LDS
        // ---- twist factors s^row / h (29-bit form), once per row when every column shares the shift
        if (row_twist) {
            const Fr* tab = p.twist + (size_t)arr * ((1ull << p.L1) + (1ull << p.L2));
            for (uint32_t rg = threadIdx.x; rg < (K << logG); rg += NTT_THREADS) {
                uint32_t t, g;
                if (t_minor) {
                    t = rg & (K - 1);
                    g = rg >> p.k;
                } else {
                    t = rg >> logG;
                    g = rg & (G - 1);
                }
                fac[(t << logG) + g] = pow2l29(tab, p.L1, row_of(t, g));
            }
            __syncthreads();
        }
        // ---- load (optionally gathering / twisting)
        if (FWD_FIRST) {
#pragma unroll
            for (uint32_t j = 0; j < NREG; ++j) {
                const uint32_t e = threadIdx.x + j * NTT_THREADS;
                uint32_t t, g, c;
                split(e, t, g, c);
                if (e >= n_el || c >= cw) continue;
                F29 f;
                if (row_twist) {
                    f = fac[(t << logG) + g];
                } else {
                    const Fr* tab = p.twist + ((size_t)arr * p.w + c0 + c) * ((1ull << p.L1) + (1ull << p.L2));
                    f = pow2l29(tab, p.L1, row_of(t, g));
                }
                lds[(((t << logG) + g) << LOGCW) + c] = f29_mul(xr[j], f);  // < 8.3 r
            }
        } else {
            for (uint32_t e = threadIdx.x; e < n_el; e += NTT_THREADS) {
                uint32_t t, g, c;
                split(e, t, g, c);
                if (c >= cw) continue;
                const uint32_t row = row_of(t, g);
                F29 v;
                if (MODE == PASS_INV_FIRST)
                    v = f29_repack_in(p.src[(size_t)brev_bits(row, p.logH) * p.w + c0 + c]);
                else
                    v = f29_repack_in(base[(size_t)row * p.w + c0 + c]);
                lds[(((t << logG) + g) << LOGCW) + c] = v;
            }
        }
        __syncthreads();
        // ---- k radix-2 stages
        const uint32_t nbf = n_el >> 1;
        for (uint32_t j = 0; j < p.k; ++j) {
            const uint32_t s = p.s0 + j;
            const uint32_t logd = DIF ? (p.k - 1 - j) : j;
            const bool trivial = DIF ? (s == p.logH - 1) : (s == 0);
            const uint32_t dmask = (1u << logd) - 1;
            // twiddle index of butterfly row i0: DIF (i0 mod H/2^(s+1)) << s, DIT (i0 mod 2^s) << (logH-1-s)
            const uint32_t tmask = DIF ? (uint32_t)((H >> (s + 1)) - 1) : ((1u << s) - 1);
            const uint32_t tshift = DIF ? s : (p.logH - 1 - s);
            for (uint32_t bf = threadIdx.x; bf < nbf; bf += NTT_THREADS) {
                const uint32_t c = bf & (CW - 1);
                const uint32_t pg = bf >> LOGCW;
                const uint32_t g = pg & (G - 1), pp = pg >> logG;
                const uint32_t t0 = ((pp >> logd) << (logd + 1)) | (pp & dmask);
                const uint32_t t1 = t0 + (1u << logd);
                const uint32_t a0 = (((t0 << logG) + g) << LOGCW) + c, a1 = (((t1 << logG) + g) << LOGCW) + c;
                const F29 a = lds[a0], b = lds[a1];
                if (trivial) {
                    lds[a0] = f29_reduce(f29_lazy2(a, b));
                    lds[a1] = f29_reduce(f29_sub16(a, b));
                    continue;
                }
                const F29 wv = f29_load48(p.tw + 3 * (size_t)((row_of(t0, g) & tmask) << tshift));
                if (DIF) {
                    lds[a0] = f29_reduce(f29_lazy2(a, b));
                    lds[a1] = f29_mul(f29_sub16(a, b), wv);
                } else {
                    const F29 bw = f29_mul(b, wv);
                    lds[a0] = f29_reduce(f29_lazy2(a, bw));
                    lds[a1] = f29_reduce(f29_sub16(a, bw));
                }
            }
            __syncthreads();
        }
        // ---- store
        const bool canon = p.canon != 0;
        for (uint32_t e = threadIdx.x; e < n_el; e += NTT_THREADS) {
            uint32_t t, g, c;
            split(e, t, g, c);
            if (c >= cw) continue;
            base[(size_t)row_of(t, g) * p.w + c0 + c] = f29_store(lds[(((t << logG) + g) << LOGCW) + c], canon);
        }
    }
}

// ark-form words -> the 29-bit Montgomery form x 2^261 mod r, canonical, packed
// in 8 words (twiddle and twist tables of k_ntt_rm)
__global__ __launch_bounds__(256) void k_to_f29form(const Fr* __restrict__ in, Fr* __restrict__ out, size_t n) {
    const size_t i = gtid();
    if (i < n) out[i] = f29_store(f29_from_fr(in[i]), true);
}

__global__ __launch_bounds__(256) void k_to_f29limbs(const Fr* __restrict__ in, uint4* __restrict__ out, size_t n) {
    const size_t i = gtid();
    if (i >= n) return;
    const F29 v = f29_repack_in(f29_store(f29_from_fr(in[i]), true));
    out[3 * i] = make_uint4(v.l[0], v.l[1], v.l[2], v.l[3]);
    out[3 * i + 1] = make_uint4(v.l[4], v.l[5], v.l[6], v.l[7]);
    out[3 * i + 2] = make_uint4(v.l[8], 0u, 0u, 0u);
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

hipError_t launch_lde(const Fr* in, Fr* X, Fr* out, size_t w, uint32_t logh, uint32_t ncosets, const uint4* tw_inv,
                      const uint4* tw_fwd, const Fr* twist, uint32_t L1, uint32_t L2, int twist_per_col,
                      hipStream_t st) {
    if (w == 0) return hipSuccess;
    // column chunk: the power of two >= min(w, 8); CW * G = 8 (256-byte row runs)
    uint32_t logCW = 0;
    while ((1u << logCW) < w && logCW < 3) ++logCW;
    const uint32_t CW = 1u << logCW;
    const uint32_t logGmax = 3 - logCW;
    const uint32_t nchunk = (uint32_t)((w + CW - 1) / CW);
    // k <= 7: a tile of <= 1024 limb-form elements (36 KiB) plus the twist factors
    const uint32_t kmax = 7;
    uint32_t ks[16], np;
    auto run = [&](bool dif, uint32_t narr, const Fr* src, Fr* dst, const uint4* tw, int first_mode,
                   bool canon_last) -> hipError_t {
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
            p.w = (uint32_t)w;
            p.nchunk = nchunk;
            p.canon = (canon_last && q + 1 == np) ? 1u : 0u;
            p.narr = narr;
            // the first forward pass loops over the cosets inside each workgroup
            const uint64_t tiles = (uint64_t)(dif && q == 0 && first_mode == PASS_FWD_FIRST ? 1 : narr) *
                                   ((1ull << logh) >> (k + logG)) * nchunk;
            // tile, plus one twist factor per row in the first forward pass
            const size_t lds = ((size_t(1) << (k + logG)) * CW + (size_t(1) << (k + logG))) * sizeof(F29);
            const int mode = q == 0 ? first_mode : PASS_INPLACE;
            const dim3 grid((unsigned)tiles), blk(256);
#define LSP_NTT_LAUNCH(DIFV, MODEV)                                                                   \
    switch (logCW) {                                                                                  \
        case 0: hipLaunchKernelGGL((k_ntt_rm<DIFV, MODEV, 0>), grid, blk, lds, st, p); break;         \
        case 1: hipLaunchKernelGGL((k_ntt_rm<DIFV, MODEV, 1>), grid, blk, lds, st, p); break;         \
        case 2: hipLaunchKernelGGL((k_ntt_rm<DIFV, MODEV, 2>), grid, blk, lds, st, p); break;         \
        default: hipLaunchKernelGGL((k_ntt_rm<DIFV, MODEV, 3>), grid, blk, lds, st, p); break;        \
    }
            if (dif) {
                if (mode == PASS_FWD_FIRST) {
                    LSP_NTT_LAUNCH(true, PASS_FWD_FIRST)
                } else {
                    LSP_NTT_LAUNCH(true, PASS_INPLACE)
                }
            } else {
                if (mode == PASS_INV_FIRST) {
                    LSP_NTT_LAUNCH(false, PASS_INV_FIRST)
                } else {
                    LSP_NTT_LAUNCH(false, PASS_INPLACE)
                }
            }
#undef LSP_NTT_LAUNCH
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
    hipError_t e = run(false, 1, in, X, tw_inv, PASS_INV_FIRST, false);
    if (e != hipSuccess) return e;
    return run(true, ncosets, X, out, tw_fwd, PASS_FWD_FIRST, true);
}

hipError_t launch_to_f29form(const Fr* in, Fr* out, size_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_to_f29form, dim3(nblocks(n, 256)), dim3(256), 0, st, in, out, n);
    return hipGetLastError();
}

hipError_t launch_to_f29limbs(const Fr* in, uint4* out, size_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_to_f29limbs, dim3(nblocks(n, 256)), dim3(256), 0, st, in, out, n);
    return hipGetLastError();
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
