// Poseidon2Bls12337<3> compression on one wave with the state spread over the
// lanes: lane 16 j + l holds limb l of state element j
// (rows 0..2; row 3 and lanes 9..15 of every row zero), every product is the
// 16-lane row product f29row_mul (fr29_row_gfx950.inc).  Same permutation and
// lazy-reduction schedule as permute3_f29 (poseidon2_f29.hpp):
//   full rounds   rows 0..2 take their S-box together (5 dependent products);
//                 t = s0 + s1 + s2 is a row sum (two permlane swaps)
//   partial rounds x, s1, s2 replicated on all four rows; x^11 = (x^4)^2 x^3
//                 with x^4 (even rows) and x^3 (odd rows) from one product
//                 (4 dependent products, as the quad form)
//   sums          carry-save: limb & mask + the lane below's limb >> 29
//                 (row_shr:1), two rounds take limbs < 2^32 to <= 2^29
//   reductions    q r from an LDS table in row layout (rqt[16 q + l]), biased
//                 as f29_reduce_qt; the quotient is taken ONE LOWER than
//                 f29_reduce_qt's (outputs in [r, 3r) instead of [0, 2r)) and
//                 entry 0 is unbiased, so the top limb of a carry-save result
//                 never goes negative (two carry-save rounds leave the biases'
//                 carries pending, which a value below 2^232 would turn into -1)
//   output        f29_to_fr's product on the row, the limbs gathered to scalars,
//                 f29_reduce and the canonical words (the one-lane code)
// Intermediate values may differ from the one-lane path's by multiples of r;
// the digest (canonical) is the same.
#pragma once
#include "poseidon2_f29.hpp"

namespace lsp {
#include "fr29_row_gfx950.inc"

namespace prow {

__device__ __forceinline__ uint32_t shr1(uint32_t x) {  // lane l <- lane l - 1 of the row, lane 0 <- 0
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t bcast8(uint32_t x) {  // lane 8 of this lane's row
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x158, 0xf, 0xf, false);
}
// rows (0,1,2,3) of a, b -> a = (a0, b0, a2, b2), b = (a1, b1, a3, b3)
__device__ __forceinline__ void swap16(uint32_t& a, uint32_t& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    a = r[0];
    b = r[1];
}
// -> a = (a0, a1, b0, b1), b = (a2, a3, b2, b3)
__device__ __forceinline__ void swap32(uint32_t& a, uint32_t& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = r[0];
    b = r[1];
}
__device__ __forceinline__ uint32_t rowsum(uint32_t x) {  // x0 + x1 + x2 + x3 on every row
    uint32_t a = x, b = x;
    swap16(a, b);
    uint32_t s = a + b, t = s;
    swap32(s, t);
    return s + t;
}
__device__ __forceinline__ uint32_t row0_all(uint32_t x) {
    uint32_t a = x, b = x;
    swap16(a, b);  // a = (x0, x0, x2, x2)
    uint32_t c = a;
    swap32(a, c);  // a = (x0, x0, x0, x0)
    return a;
}
__device__ __forceinline__ uint32_t row1_all(uint32_t x) {
    uint32_t a = x, b = x;
    swap16(a, b);  // b = (x1, x1, x3, x3)
    uint32_t c = b;
    swap32(b, c);
    return b;
}
__device__ __forceinline__ uint32_t row2_all(uint32_t x) {
    uint32_t a = x, b = x;
    swap32(a, b);  // b = (x2, x3, x2, x3)
    uint32_t c = b;
    swap16(b, c);  // b = (x2, x2, x2, x2)
    return b;
}

struct Lane {
    F29RowK K;      // the row product's per-lane constants
    uint32_t l;     // limb index (lane % 16)
    uint32_t row;   // lane / 16
    bool hi9;       // l >= 9
};

// carry-save normalisation of a limb-wise sum (limbs < 2^32): limbs 0..7 <= 2^29
__device__ __forceinline__ uint32_t rnorm(uint32_t v, const Lane& L) {
#pragma unroll
    for (int k = 0; k < 2; ++k) v = (v & L.K.maskl) + shr1(v >> 29);
    return L.hi9 ? 0u : v;
}

// the workgroup's LDS: the row-layout reduction table rqt[16 q + l] (f29_reduce_qt's
// biased limb l of q r) and the row product's per-lane constants, indexed by lane
struct RowLds {
    uint32_t rqt[16 * F29_QTAB_N];
    uint32_t ptab[32];  // [8 + d] = p29(d) for d = 1..8, else 0: lane l's P[k] = ptab[8 + l - k]
    uint32_t c0[16];    // c29(l), 0 beyond limb 8
    uint32_t cto[16];   // limb l of f29_to_fr's constant 2^256 mod r (the product by it is x 2^-5)
};

__device__ __forceinline__ void row_lds_init(RowLds* t) {
    for (uint32_t q = threadIdx.x; q < F29_QTAB_N; q += blockDim.x) {
        uint32_t Q[9];
        uint64_t c = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint64_t v = (uint64_t)q * p29(i) + c;
            Q[i] = (uint32_t)v & F29_MASK;
            c = v >> 29;
        }
        Q[8] = (uint32_t)((uint64_t)q * p29(8) + c);
        // entry 0 is all zero, not the biased zero: a small value passes through
        // with non-negative limbs (the biases' carries would leave its top limb at -1)
        uint32_t* e = t->rqt + 16 * q;
        const uint32_t b = q ? 2u : 0u;
        e[0] = q ? (1u << 30) - Q[0] : 0u;
#pragma unroll
        for (int i = 1; i < 8; ++i) e[i] = q ? (1u << 30) - b - Q[i] : 0u;
        e[8] = 0u - b - Q[8];
#pragma unroll
        for (int i = 9; i < 16; ++i) e[i] = 0u;
    }
    constexpr uint32_t TO[9] = {0x1ffffff3u, 0x8e3ffffu, 0x1ffffc9fu, 0xfea1edfu, 0xfee725u,
                                0xabaa896u,  0xa745b60u, 0x6457773u,  0xd4bdau};  // f29_to_fr's c
    for (uint32_t i = threadIdx.x; i < 32; i += blockDim.x) {
        uint32_t v = 0;
#pragma unroll
        for (int d = 1; d <= 8; ++d) v = i == 8u + d ? p29(d) : v;
        t->ptab[i] = v;
        if (i < 16) {
            uint32_t c = 0, o = 0;
#pragma unroll
            for (int l = 0; l < 9; ++l) {
                c = i == (uint32_t)l ? c29(l) : c;
                o = i == (uint32_t)l ? TO[l] : o;
            }
            t->c0[i] = c;
            t->cto[i] = o;
        }
    }
}

__device__ __forceinline__ Lane row_lane(const RowLds* t) {
    Lane L;
    const uint32_t lane = threadIdx.x & 63u;
    L.l = lane & 15u;
    L.row = lane >> 4;
    L.hi9 = L.l >= 9;
    L.K.c0 = t->c0[L.l];
#pragma unroll
    for (int k = 0; k < 9; ++k) L.K.P[k] = t->ptab[8 + L.l - k];
    L.K.maskl = L.l == 8 ? 0xffffffffu : F29_MASK;
    return L;
}

// this lane's table entry for v - (q - 1) r (q as f29_reduce_qt; v < 64 r, limbs
// < 2.4 2^30): rnorm(v + entry) is in [r, 3r) for q >= 2, v itself below -- the
// result's top limb is never negative (lower limbs carry-save, <= 2^29)
__device__ __forceinline__ uint32_t rq_entry(uint32_t v, const uint32_t* __restrict__ rqt, const Lane& L) {
    uint32_t q = __umulhi(bcast8(v), 0xdb651d12u) >> 20;
    if (!LSP_BOUNDS(q < F29_QTAB_N)) q = 0;
    q = q ? q - 1 : 0u;
    return rqt[16 * q + L.l];
}
__device__ __forceinline__ uint32_t rreduce(uint32_t v, const uint32_t* __restrict__ rqt, const Lane& L) {
    return rnorm(v + rq_entry(v, rqt, L), L);
}

__device__ __forceinline__ uint32_t rmul(uint32_t a, uint32_t b, const Lane& L) { return f29row_mul(a, b, L.K); }

template <uint32_t D>
__device__ __forceinline__ uint32_t sbox(uint32_t x, const Lane& L) {
    const uint32_t x2 = rmul(x, x, L);
    const uint32_t x4 = rmul(x2, x2, L);
    const uint32_t x8 = rmul(x4, x4, L);
    if (D == 11) return rmul(rmul(x8, x2, L), x, L);
    return rmul(rmul(x8, x8, L), x, L);  // x^17
}

// this lane's limb of the ark-form Fr at p as f29_from_fr_lazy (X 2^5, < 32 r)
__device__ __forceinline__ uint32_t load_limb(const Fr* p, const Lane& L) {
    if (L.hi9) return 0u;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
    const uint32_t b = 29 * L.l + 27, W = b >> 5;  // bits [29 l - 5, 29 l + 24) of X, one word up
    const uint32_t lo = W ? w[W - 1] : 0u, hi = W < 8 ? w[W] : 0u;
    const uint32_t v = __builtin_amdgcn_alignbit(hi, lo, b & 31);
    return L.l < 8 ? v & F29_MASK : v;
}

// this lane's limb of constant k (0 for lanes 9..15)
__device__ __forceinline__ uint32_t rc_limb(const F29* __restrict__ rc29, uint32_t k, const Lane& L) {
    return L.hi9 ? 0u : rc29[k].l[L.l];
}

// compress(left, right) for the wave (S-box degree D = 11 or 17, default
// linear layers).  Every lane of the wave must be active; the tables published
// (row_lds_init + barrier).
template <uint32_t D>
__device__ __forceinline__ Fr compress_row(const Fr* left, const Fr* right, const F29* __restrict__ rc29, uint32_t rf,
                                           uint32_t rp, const RowLds* __restrict__ tab) {
    const Lane L = row_lane(tab);
    const uint32_t* rqt = tab->rqt;
    const uint32_t half = rf / 2;
    const F29* ini = rc29;
    const F29* ter = rc29 + 3 * half;
    const F29* itl = rc29 + 6 * half;
    // state: row j = s_j (row 3 zero)
    uint32_t S = L.row == 0 ? load_limb(left, L) : L.row == 1 ? load_limb(right, L) : 0u;
    S = rreduce(S, rqt, L);
    uint32_t T = rowsum(S);
    const bool live = L.row < 3;
    uint32_t C = live ? rc_limb(ini, L.row, L) : 0u;
    for (uint32_t r = 0; r < half; ++r) {
        const uint32_t x = rnorm(S + C + T, L);
        C = live && r + 1 < half ? rc_limb(ini, 3 * (r + 1) + L.row, L) : 0u;
        const uint32_t y = sbox<D>(x, L);
        S = live ? y : 0u;
        T = rowsum(S);
    }
    // into the partial rounds: x = s0 + c + t, s1 and s2 reduced; replicated on every row
    const uint32_t W = S + T;
    uint32_t Ci = rp ? rc_limb(itl, 0, L) : 0u;
    uint32_t X = row0_all(rnorm(W + Ci, L));
    const uint32_t R = rreduce(W, rqt, L);
    uint32_t S1 = row1_all(R), S2 = row2_all(R);
    const bool odd = L.row & 1u;
    // s1 and s2's reductions finish in the next round, after its first product,
    // so their table reads are in flight behind it: s_j = rnorm(v_j + e_j)
    uint32_t v1 = S1, v2 = S2, e1 = 0, e2 = 0;
    for (uint32_t r = 0; r < rp; ++r) {
        Ci = r + 1 < rp ? rc_limb(itl, r + 1, L) : 0u;
        const uint32_t x2 = rmul(X, X, L);
        S1 = rnorm(v1 + e1, L);
        S2 = rnorm(v2 + e2, L);
        uint32_t y;
        if (D == 11) {
            uint32_t a = rmul(x2, odd ? X : x2, L);  // even rows x^4, odd rows x^3
            uint32_t b = a;
            swap16(a, b);  // a = x^4, b = x^3 on every row
            y = rmul(rmul(a, a, L), b, L);
        } else {
            const uint32_t x4 = rmul(x2, x2, L);
            const uint32_t x8 = rmul(x4, x4, L);
            y = rmul(rmul(x8, x8, L), X, L);  // x^17
        }
        const uint32_t u = y + S1 + S2;  // carry-free, limbs <= 3 2^29 + 2
        v1 = S1 + u;
        v2 = S2 + S2 + u;
        e1 = rq_entry(v1, rqt, L);
        e2 = rq_entry(v2, rqt, L);
        X = rnorm(y + Ci + u, L);
    }
    S1 = rnorm(v1 + e1, L);
    S2 = rnorm(v2 + e2, L);
    S = L.row == 0 ? X : L.row == 1 ? S1 : L.row == 2 ? S2 : 0u;
    T = 0;
    C = live ? rc_limb(ter, L.row, L) : 0u;
    for (uint32_t r = 0; r < half; ++r) {
        const uint32_t x = rnorm(S + C + T, L);
        C = live && r + 1 < half ? rc_limb(ter, 3 * (r + 1) + L.row, L) : 0u;
        const uint32_t y = sbox<D>(x, L);
        S = live ? y : 0u;
        T = rowsum(S);
    }
    // f29_to_fr of row 0's s0 + t: the product by its constant on the row, then
    // the limbs to scalars, f29_reduce (< 2 r, normalised), canonical words
    const uint32_t y = rmul(rnorm(S + T, L), tab->cto[L.l], L);
    F29 o;
#pragma unroll
    for (int i = 0; i < 9; ++i) o.l[i] = __builtin_amdgcn_readlane(y, i);
    return fr_reduce_once(f29_repack_out(f29_reduce(o)));
}

}  // namespace prow
}  // namespace lsp
