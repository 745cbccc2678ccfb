// Quotient evaluation over the LDE domain: p3-uni-stark quotient_values with
// ProverConstraintFolder, running LineaAIR::eval (air/src/lib.rs:47-167) for
// every point of the quotient coset GEN * H_Q.
//
// The AIR is the int32 AirConfig descriptor of include/lsp.h, interpreted
// with wave-uniform control flow (every lane walks the same configs); the
// folder's accumulation acc = acc*alpha + C_j (Horner, U10) runs in the
// constraint order of eval.  Row `local` is LDE row bitrev_Q(i) and `next`
// is bitrev_Q((i + 2^log_q) mod Q) (get_evaluations_on_domain +
// vertically_packed_row_pair).
#include <cstdlib>

#include "fr29.hpp"
#include "k_common.hpp"
#include "kernels.hpp"

namespace lsp {

namespace {
// The constraint arithmetic runs on the 29-bit-limb product (fr29.hpp; ~2x the
// 8 x 32-bit product's rate): every trace value and constant enters in the
// 29-bit form (x 2^261: a repack and a cheap reduction from the ark form),
// sums and differences leave through the LDS-table reduction (< 2 r,
// normalised), products stay as the multiplier leaves them (normalised,
// < 8.92 r for inputs < 20 r), and the quotient value leaves canonical in the
// ark form.  Bounds: add / sub inputs < 20 r give < 40 r with limbs < 1.5 2^30
// (f29_reduce_qt takes < 64 r, limbs < 2.41 2^30); f29_sub16 takes a
// subtrahend < 16 r.
struct Q29 {
    const uint4* qt;
    __device__ __forceinline__ F29 add(const F29& a, const F29& b) const { return f29_reduce_qt(f29_lazy2(a, b), qt); }
    __device__ __forceinline__ F29 sub(const F29& a, const F29& b) const { return f29_reduce_qt(f29_sub16(a, b), qt); }
    __device__ __forceinline__ F29 mul(const F29& a, const F29& b) const { return f29_mul(a, b); }
};

// column k of a row (the descriptor's ids are checked against the width on
// the host, Air::parse; the debug build checks them again here)
__device__ __forceinline__ F29 ld29(const Fr* __restrict__ row, int32_t k, uint32_t w) {
    return LSP_BOUNDS(k >= 0 && (uint32_t)k < w) ? f29_from_fr(row[k]) : f29_zero();
}

__device__ __forceinline__ F29 horner(const Q29& F, const Fr* __restrict__ row, const int32_t* __restrict__ ids,
                                      int32_t n, const F29& a, uint32_t w) {
    F29 acc = f29_zero();
    for (int32_t k = 0; k < n; ++k) acc = F.add(F.mul(acc, a), ld29(row, ids[k], w));
    return acc;
}

__global__ __launch_bounds__(256) void k_selector_denoms(const Fr* __restrict__ tabQ, uint32_t L1, Fr gen,
                                                         Fr wh_inv, size_t n, uint64_t i0, uint32_t log_step,
                                                         Fr* __restrict__ den) {
    const size_t m = gtid();
    if (m >= n) return;
    const uint64_t i = i0 + ((uint64_t)m << log_step);
    const Fr x = fr_mul(gen, pow2l(tabQ, L1, i));
    den[m] = fr_mul(fr_sub(x, fr_one()), fr_sub(x, wh_inv));
}

// one constraint value of thread t, limb-planar (QuotientArgs::cons)
__device__ __forceinline__ void st_cons(const QuotientArgs& a, uint32_t j, size_t t, size_t n, const F29& v) {
    if (!LSP_BOUNDS(j < a.ncons)) return;
    uint32_t* c = a.cons + (size_t)j * 9 * n + t;
#pragma unroll
    for (int l = 0; l < 9; ++l) c[(size_t)l * n] = v.l[l];
}

// EARLY: write the constraint values (QuotientArgs::cons) instead of folding them
template <bool EARLY>
__global__ __launch_bounds__(256) void k_quotient(QuotientArgs a) {
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt's table
    f29_qtab_init(qt);
    __syncthreads();
    const Q29 F{qt};
    const size_t t = gtid();
    const size_t Q = 1ull << a.logQ;
    const size_t npts = a.n ? a.n : Q;
    if (t >= npts) return;  // n = Q >> log_step points
    const size_t tcons = t;  // (the lookup loop below names its table index t)
    // Row order: thread t evaluates point m = bitrev(t), whose row bitrev_Q(i)
    // is row0 + t, so a wave reads 64 adjacent LDE rows (and their
    // successors).  In point order it read rows Q/64 apart: with the C3
    // trace's 5.9 KB rows their lines left the L2 before the lane came back
    // for the next columns (2^20 x 184: 63.5 -> 36.7 ms), and with narrow
    // rows past the caches' size every row is a DRAM page miss (round 3:
    // 2^22 x 8 5.7 -> 3.9 ms).  Point order (coalesced inv_den reads and out
    // writes) remains for A/B runs (row_order = 0).
    const size_t m = a.row_order ? brev_bits(t, a.logQ - a.log_step) : t;
    const uint64_t i = a.i0 + ((uint64_t)m << a.log_step);
    const uint32_t qmask = (1u << a.log_q) - 1;
    const F29 one = f29_from_fr(fr_one());
    const Fr x = fr_mul(a.gen, pow2l(a.tabQ, a.L1, i));
    const Fr xm1 = fr_sub(x, fr_one());
    const Fr xml = fr_sub(x, a.wh_inv);
    const F29 zh = f29_from_fr(a.zh[i & qmask]), inv_den = f29_from_fr(a.inv_den[m]);
    const F29 xml29 = f29_from_fr(xml);
    const F29 first = F.mul(zh, F.mul(xml29, inv_den));              // Z_H / (x - 1)
    const F29 last = F.mul(zh, F.mul(f29_from_fr(xm1), inv_den));  // Z_H / (x - w^-1)
    const F29 trans = xml29;                                         // x - w^-1
    const uint64_t lrow = brev_bits(i, a.logQ) - a.row0;
    const uint64_t nrow = brev_bits((i + (1ull << a.log_q)) & (Q - 1), a.logQ) - (a.lde_next ? a.row0_next : a.row0);
    // the rows this rank holds (lde_rows = 0: not given, unchecked)
    if (!LSP_BOUNDS(a.lde_rows == 0 || (lrow < a.lde_rows && nrow < (a.lde_next ? a.lde_next_rows : a.lde_rows))))
        return;
    const Fr* loc = a.lde + lrow * a.w;
    const Fr* nxt = (a.lde_next ? a.lde_next : a.lde) + nrow * a.w;
    const F29 ap = f29_from_fr(a.pub_alpha), dl = f29_from_fr(a.pub_delta), al = f29_from_fr(a.alpha);
    F29 acc = f29_zero();
    uint32_t ncw = 0;  // constraints written (EARLY)
#define PUSH(X)                                     \
    do {                                            \
        if constexpr (EARLY)                        \
            st_cons(a, ncw++, tcons, npts, (X));    \
        else                                        \
            acc = F.add(F.mul(acc, al), (X));       \
    } while (0)
    const int32_t* d = a.air;
    int32_t p = 0;
    const int32_t ncfg = d[p++];
    for (int32_t c = 0; c < ncfg; ++c) {
        const int32_t type = d[p++];
        if (type == 1) {  // AirPermutationConfig: air/src/lib.rs:116-167
            const int32_t na = d[p++], nb = d[p++];
            const int32_t* aid = d + p;
            p += na;
            const int32_t* bid = d + p;
            p += nb;
            const int32_t binv = d[p++], chk = d[p++];
            const F29 a_l = F.add(horner(F, loc, aid, na, ap, a.w), dl);
            const F29 b_l = F.add(horner(F, loc, bid, nb, ap, a.w), dl);
            const F29 lbinv = ld29(loc, binv, a.w), lchk = ld29(loc, chk, a.w);
            PUSH(F.sub(F.mul(b_l, lbinv), one));
            PUSH(F.mul(first, F.sub(lchk, F.mul(a_l, lbinv))));
            const F29 a_n = F.add(horner(F, nxt, aid, na, ap, a.w), dl);
            PUSH(F.mul(trans, F.sub(ld29(nxt, chk, a.w), F.mul(F.mul(lchk, a_n), ld29(nxt, binv, a.w)))));
            PUSH(F.mul(last, F.sub(lchk, one)));
        } else {  // AirLookupConfig: air/src/lib.rs:57-114
            const int32_t na = d[p++];
            const int32_t* aid = d + p;
            p += na;
            const int32_t nt = d[p++], nbc = d[p++];
            const int32_t* bid = d + p;
            p += nt * nbc;
            const int32_t afil = d[p++];
            const int32_t* bfil = d + p;
            p += nt;
            const int32_t ainv = d[p++];
            const int32_t* binv = d + p;
            p += nt;
            const int32_t* occ = d + p;
            p += nt;
            const int32_t chk = d[p++];
            const F29 a_l = F.add(horner(F, loc, aid, na, ap, a.w), dl);
            const F29 lainv = ld29(loc, ainv, a.w);
            PUSH(F.sub(F.mul(a_l, lainv), one));
            F29 lc = F.mul(ld29(loc, afil, a.w), lainv);
            F29 nc = F.mul(ld29(nxt, afil, a.w), ld29(nxt, ainv, a.w));
            for (int32_t t = 0; t < nt; ++t) {
                const F29 b_l = F.add(horner(F, loc, bid + t * nbc, nbc, ap, a.w), dl);
                const F29 lbinv = ld29(loc, binv[t], a.w);
                PUSH(F.sub(F.mul(b_l, lbinv), one));
                lc = F.sub(lc, F.mul(F.mul(ld29(loc, bfil[t], a.w), ld29(loc, occ[t], a.w)), lbinv));
                nc = F.sub(nc, F.mul(F.mul(ld29(nxt, bfil[t], a.w), ld29(nxt, occ[t], a.w)), ld29(nxt, binv[t], a.w)));
            }
            const F29 lchk = ld29(loc, chk, a.w);
            PUSH(F.mul(first, F.sub(lchk, lc)));
            PUSH(F.mul(trans, F.sub(F.sub(ld29(nxt, chk, a.w), lchk), nc)));
            PUSH(F.mul(last, lchk));
        }
    }
#undef PUSH
    if constexpr (!EARLY) a.out[m] = f29_to_fr_qt(F.mul(acc, f29_from_fr(a.inv_zh[i & qmask])), qt);
}

// the fold of the values k_quotient<true> wrote: thread t reads its own
// (coalesced) and writes point m as k_quotient<false> would
__global__ __launch_bounds__(256) void k_quotient_fold(QuotientArgs a) {
    __shared__ uint4 qt[3 * F29_QTAB_N];
    f29_qtab_init(qt);
    __syncthreads();
    const Q29 F{qt};
    const size_t t = gtid();
    const size_t npts = a.n ? a.n : (1ull << a.logQ);
    if (t >= npts) return;
    const size_t m = a.row_order ? brev_bits(t, a.logQ - a.log_step) : t;
    const uint64_t i = a.i0 + ((uint64_t)m << a.log_step);
    const uint32_t qmask = (1u << a.log_q) - 1;
    const F29 al = f29_from_fr(a.alpha);
    F29 acc = f29_zero();
    for (uint32_t j = 0; j < a.ncons; ++j) {
        const uint32_t* c = a.cons + (size_t)j * 9 * npts + t;
        F29 v;
#pragma unroll
        for (int l = 0; l < 9; ++l) v.l[l] = c[(size_t)l * npts];
        acc = F.add(F.mul(acc, al), v);
    }
    a.out[m] = f29_to_fr_qt(F.mul(acc, f29_from_fr(a.inv_zh[i & qmask])), qt);
}
}  // namespace

hipError_t launch_selector_denoms(const Fr* tabQ, uint32_t L1, Fr gen, Fr wh_inv, size_t n, Fr* den,
                                  hipStream_t st, uint64_t i0, uint32_t log_step) {
    hipLaunchKernelGGL(k_selector_denoms, dim3(nblocks(n, 256)), dim3(256), 0, st, tabQ, L1, gen, wh_inv, n, i0,
                       log_step, den);
    return hipGetLastError();
}

// Thread order: LDE row order (LSP_QUOTIENT_ORDER=point: point order; read per
// call).  Row order measured faster at every size (profiles/r03x_quotient_order.txt:
// 2^19 x 8 0.475 -> 0.45 ms, 2^22 x 8 5.7 -> 3.9 ms, rank 0 of 2^26 over 8 ranks
// 60 -> 26 ms): in point order a wave's 64 rows are Q/64 apart, and past the
// caches' size every row is a DRAM page miss.
static QuotientArgs with_order(const QuotientArgs& a) {
    QuotientArgs b = a;
    b.row_order = 1;
    if (const char* e = std::getenv("LSP_QUOTIENT_ORDER")) {
        if (e[0] == 'r') b.row_order = 1;
        if (e[0] == 'p') b.row_order = 0;
    }
    return b;
}

hipError_t launch_quotient(const QuotientArgs& a, hipStream_t st) {
    const size_t n = a.n ? a.n : (1ull << a.logQ);
    const QuotientArgs b = with_order(a);
    if (a.cons)
        hipLaunchKernelGGL(k_quotient<true>, dim3(nblocks(n, 256)), dim3(256), 0, st, b);
    else
        hipLaunchKernelGGL(k_quotient<false>, dim3(nblocks(n, 256)), dim3(256), 0, st, b);
    return hipGetLastError();
}

hipError_t launch_quotient_fold(const QuotientArgs& a, hipStream_t st) {
    if (!a.cons) return hipErrorInvalidValue;
    const size_t n = a.n ? a.n : (1ull << a.logQ);
    hipLaunchKernelGGL(k_quotient_fold, dim3(nblocks(n, 256)), dim3(256), 0, st, with_order(a));
    return hipGetLastError();
}

}  // namespace lsp

LSP_BOUNDS_READER(k_quotient)
