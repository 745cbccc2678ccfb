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
#include "k_common.hpp"
#include "kernels.hpp"

namespace lsp {

namespace {
__device__ __forceinline__ Fr horner(const Fr* __restrict__ row, const int32_t* __restrict__ ids, int32_t n,
                                     const Fr& a) {
    Fr acc = fr_zero();
    for (int32_t k = 0; k < n; ++k) acc = fr_add(fr_mul(acc, a), row[ids[k]]);
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

__global__ __launch_bounds__(256) void k_quotient(QuotientArgs a) {
    const size_t t = gtid();
    const size_t Q = 1ull << a.logQ;
    if (t >= (a.n ? a.n : Q)) return;  // n = Q >> log_step points
    // Wide rows: thread t evaluates point m = bitrev(t), whose row bitrev_Q(i)
    // is row0 + t, so a wave reads 64 adjacent LDE rows (and their
    // successors).  In point order it read rows Q/64 apart, and with the C3
    // trace's 5.9 KB rows their lines left the L2 before the lane came back
    // for the next columns (2^20 x 184: 63.5 -> 36.7 ms).  Narrow rows keep
    // point order (coalesced inv_den reads and out writes; 2^19 x 8 is ~5 %
    // faster that way).
    const size_t m = a.w >= 32 ? brev_bits(t, a.logQ - a.log_step) : t;
    const uint64_t i = a.i0 + ((uint64_t)m << a.log_step);
    const uint32_t qmask = (1u << a.log_q) - 1;
    const Fr one = fr_one();
    const Fr x = fr_mul(a.gen, pow2l(a.tabQ, a.L1, i));
    const Fr xm1 = fr_sub(x, one);
    const Fr xml = fr_sub(x, a.wh_inv);
    const Fr zh = a.zh[i & qmask];
    const Fr first = fr_mul(zh, fr_mul(xml, a.inv_den[m]));  // Z_H / (x - 1)
    const Fr last = fr_mul(zh, fr_mul(xm1, a.inv_den[m]));   // Z_H / (x - w^-1)
    const Fr trans = xml;                                    // x - w^-1
    const Fr* loc = a.lde + (brev_bits(i, a.logQ) - a.row0) * a.w;
    const Fr* nxt = a.lde + (brev_bits((i + (1ull << a.log_q)) & (Q - 1), a.logQ) - a.row0) * a.w;
    const Fr ap = a.pub_alpha, dl = a.pub_delta, al = a.alpha;
    Fr acc = fr_zero();
#define PUSH(X) acc = fr_add(fr_mul(acc, al), (X))
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
            const Fr a_l = fr_add(horner(loc, aid, na, ap), dl);
            const Fr b_l = fr_add(horner(loc, bid, nb, ap), dl);
            PUSH(fr_sub(fr_mul(b_l, loc[binv]), one));
            PUSH(fr_mul(first, fr_sub(loc[chk], fr_mul(a_l, loc[binv]))));
            const Fr a_n = fr_add(horner(nxt, aid, na, ap), dl);
            PUSH(fr_mul(trans, fr_sub(nxt[chk], fr_mul(fr_mul(loc[chk], a_n), nxt[binv]))));
            PUSH(fr_mul(last, fr_sub(loc[chk], one)));
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
            const Fr a_l = fr_add(horner(loc, aid, na, ap), dl);
            PUSH(fr_sub(fr_mul(a_l, loc[ainv]), one));
            Fr lc = fr_mul(loc[afil], loc[ainv]);
            Fr nc = fr_mul(nxt[afil], nxt[ainv]);
            for (int32_t t = 0; t < nt; ++t) {
                const Fr b_l = fr_add(horner(loc, bid + t * nbc, nbc, ap), dl);
                PUSH(fr_sub(fr_mul(b_l, loc[binv[t]]), one));
                lc = fr_sub(lc, fr_mul(fr_mul(loc[bfil[t]], loc[occ[t]]), loc[binv[t]]));
                nc = fr_sub(nc, fr_mul(fr_mul(nxt[bfil[t]], nxt[occ[t]]), nxt[binv[t]]));
            }
            PUSH(fr_mul(first, fr_sub(loc[chk], lc)));
            PUSH(fr_mul(trans, fr_sub(fr_sub(nxt[chk], loc[chk]), nc)));
            PUSH(fr_mul(last, loc[chk]));
        }
    }
#undef PUSH
    a.out[m] = fr_mul(acc, a.inv_zh[i & qmask]);
}
}  // namespace

hipError_t launch_selector_denoms(const Fr* tabQ, uint32_t L1, Fr gen, Fr wh_inv, size_t n, Fr* den,
                                  hipStream_t st, uint64_t i0, uint32_t log_step) {
    hipLaunchKernelGGL(k_selector_denoms, dim3(nblocks(n, 256)), dim3(256), 0, st, tabQ, L1, gen, wh_inv, n, i0,
                       log_step, den);
    return hipGetLastError();
}

hipError_t launch_quotient(const QuotientArgs& a, hipStream_t st) {
    const size_t n = a.n ? a.n : (1ull << a.logQ);
    hipLaunchKernelGGL(k_quotient, dim3(nblocks(n, 256)), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace lsp
