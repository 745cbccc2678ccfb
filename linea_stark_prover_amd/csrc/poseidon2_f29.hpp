// Poseidon2Bls12337<3> on the 29-bit-limb representation (fr29.hpp).
// Same permutation as poseidon2.hpp (U1-U3 conventions); only the arithmetic
// representation differs.  Lazy-reduction bounds (r = the field modulus;
// "normalised" = limbs 0..7 < 2^29; a product of inputs < K r is normalised
// and < (8 + 0.0023 K^2) r, fr29.hpp):
//   S-box inputs are normalised (one carry-propagating add) and < 86 r
//     (< 2^259), outputs < 9.7 r (fixed point of the bounds below);
//   the external layer's t = s0 + s1 + s2 is a limb-wise sum (no carries)
//     folded into the next S-box input with the round constant: inputs
//     < 4 Y + 2 inside a permutation (Y = the S-box output bound), < 8 Y + 6
//     at the start of a sponge permutation (s2 carries over);
//   partial rounds: u = y + s1 + s2 carry-free (limbs < 1.5 2^30, < Y + 4 r),
//     s1 = reduce(s1 + u), s2 = reduce(2 s2 + u): limb-wise sums (< Y + 8 r,
//     limbs < 2.5 2^30) into the LDS-table reduction f29_reduce_qt (`qt`,
//     valid below 64 r with limbs below 3 2^30, tests/test_f29_bounds.py), so
//     s1 and s2 stay < 2 r for any number of partial rounds; the next S-box
//     input y + c + u (one carry-propagating add) is < 2 Y + 5 r;
//   the output state is normalised and < 4 Y.
#pragma once
#include "fr29.hpp"

namespace lsp {

template <uint32_t D>
__device__ __forceinline__ F29 sbox29(const F29& x) {
    const F29 x2 = f29_sqr(x);
    const F29 x4 = f29_sqr(x2);
    const F29 x8 = f29_sqr(x4);
    if (D == 11) return f29_mul(f29_mul(x8, x2), x);
    return f29_mul(f29_sqr(x8), x);  // x^17
}


// The partial rounds: the internal layer's sum u stays carry-free and only s1
// and s2 are reduced (header).  LANES: 1 (one state per lane) or 2 / 4
// (cooperative S-box).
template <uint32_t D, int LANES>
__device__ __forceinline__ F29 partial_rounds_f29(F29 x, F29& s1, F29& s2, const F29* __restrict__ itl, uint32_t rp,
                                                  const uint4* __restrict__ qt);

// rc29: round constants in F29 form, new_from_rng order (initial external
// [rf/2][3], terminal external [rf/2][3], internal [rp])
template <uint32_t D>
__device__ __forceinline__ void permute3_f29(F29& s0, F29& s1, F29& s2, const F29* __restrict__ rc29, uint32_t rf,
                                             uint32_t rp, const uint4* __restrict__ qt) {
    const uint32_t half = rf / 2;
    const F29* ini = rc29;
    const F29* ter = rc29 + 3 * half;
    const F29* itl = rc29 + 6 * half;
    // t: the pending external layer (s_i + t), applied at the next S-box input
    F29 t = f29_lazy3(s0, s1, s2);
    for (uint32_t r = 0; r < half; ++r) {
        s0 = sbox29<D>(f29_add(f29_lazy2(s0, ini[3 * r + 0]), t));
        s1 = sbox29<D>(f29_add(f29_lazy2(s1, ini[3 * r + 1]), t));
        s2 = sbox29<D>(f29_add(f29_lazy2(s2, ini[3 * r + 2]), t));
        t = f29_lazy3(s0, s1, s2);
    }
    // x: the next partial-round S-box input (s0 + round constant)
    F29 x = rp ? f29_add(f29_lazy2(s0, itl[0]), t) : f29_add(s0, t);
    s1 = f29_reduce_qt(f29_lazy2(s1, t), qt);  // < 38.8 r, limbs < 2^31
    s2 = f29_reduce_qt(f29_lazy2(s2, t), qt);
    x = partial_rounds_f29<D, 1>(x, s1, s2, itl, rp, qt);
    s0 = x;
    t = f29_zero();
    for (uint32_t r = 0; r < half; ++r) {
        s0 = sbox29<D>(f29_add(f29_lazy2(s0, ter[3 * r + 0]), t));
        s1 = sbox29<D>(f29_add(f29_lazy2(s1, ter[3 * r + 1]), t));
        s2 = sbox29<D>(f29_add(f29_lazy2(s2, ter[3 * r + 2]), t));
        t = f29_lazy3(s0, s1, s2);
    }
    s0 = f29_add(s0, t);
    s1 = f29_add(s1, t);
    s2 = f29_add(s2, t);
}

// ---- quad-cooperative permutation, for launches narrower than the chip.
// One state lives in the 4 lanes of a DPP quad, replicated; in a full round
// lane j (< 3; lane 3 mirrors lane 2) computes only S-box j and the quad
// exchanges the three results with quad_perm broadcasts, so a full round costs
// one S-box instead of three.  Partial rounds run redundantly in every lane.
// Critical path: rf + rp S-boxes instead of 3 rf + rp (e.g. 30 vs 46); every
// lane of the quad must be active.
__device__ __forceinline__ uint32_t quad_bcast(uint32_t x, int q) {
    switch (q) {
        case 0:
            return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x00, 0xf, 0xf, false);
        case 1:
            return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x55, 0xf, 0xf, false);
        default:
            return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xaa, 0xf, 0xf, false);
    }
}

// the same within lane pairs (0,1), (2,3) of a quad: quad_perm [0,0,2,2] / [1,1,3,3]
__device__ __forceinline__ uint32_t pair_bcast(uint32_t x, int q) {
    return q == 0 ? (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xa0, 0xf, 0xf, false)
                  : (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xf5, 0xf, 0xf, false);
}

// lane q (0 or 1) of this lane's group (a pair when LANES == 2, else a quad)
template <int LANES>
__device__ __forceinline__ uint32_t group_bcast(uint32_t x, int q) {
    return LANES == 2 ? pair_bcast(x, q) : quad_bcast(x, q);
}

__device__ __forceinline__ F29 f29_sel3(uint32_t j, const F29& a, const F29& b, const F29& c) {
    // branch-free: masks instead of ?: (which the compiler turns into exec-mask branches)
    const uint32_t m0 = 0u - (uint32_t)(j == 0), m1 = 0u - (uint32_t)(j == 1), m2 = ~(m0 | m1);
    F29 r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.l[i] = (a.l[i] & m0) | (b.l[i] & m1) | (c.l[i] & m2);
    return r;
}

// one full round on a quad, with the pending external layer t of the
// previous round folded into the S-box input; returns the new pending t
template <uint32_t D>
__device__ __forceinline__ F29 full_round_coop(F29& s0, F29& s1, F29& s2, const F29& t, const F29* __restrict__ c,
                                               uint32_t j) {
    const F29 in = f29_sel3(j, f29_lazy2(s0, c[0]), f29_lazy2(s1, c[1]), f29_lazy2(s2, c[2]));
    const F29 x = sbox29<D>(f29_add(in, t));
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        s0.l[i] = quad_bcast(x.l[i], 0);
        s1.l[i] = quad_bcast(x.l[i], 1);
        s2.l[i] = quad_bcast(x.l[i], 2);
    }
    return f29_lazy3(s0, s1, s2);
}

// partial-round S-box on a quad: x^11 = x^8 x^3 with x^4 (lane 0) and x^3
// (lane 1) in parallel after x^2 -- four sequential products instead of five
template <uint32_t D, int LANES = 4>
__device__ __forceinline__ F29 sbox29_coop(const F29& x) {
    if (D != 11) return sbox29<D>(x);
    const F29 x2 = f29_sqr(x);
    const uint32_t odd = 0u - (threadIdx.x & 1u);
    F29 sel;
#pragma unroll
    for (int i = 0; i < 9; ++i) sel.l[i] = (x.l[i] & odd) | (x2.l[i] & ~odd);
    const F29 y = f29_mul(x2, sel);  // even lane: x^4, odd lane: x^3
    F29 x4, x3;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        x4.l[i] = group_bcast<LANES>(y.l[i], 0);
        x3.l[i] = group_bcast<LANES>(y.l[i], 1);
    }
    return f29_mul(f29_sqr(x4), x3);
}


template <uint32_t D, int LANES>
__device__ __forceinline__ F29 partial_rounds_f29(F29 x, F29& s1, F29& s2, const F29* __restrict__ itl, uint32_t rp,
                                                  const uint4* __restrict__ qt) {
    auto sb = [](const F29& v) {
        if constexpr (LANES == 1)
            return sbox29<D>(v);
        else
            return sbox29_coop<D, LANES>(v);
    };
    for (uint32_t r = 0; r < rp; ++r) {
        const F29 y = sb(x);
        const F29 u = f29_lazy3(y, s1, s2);              // carry-free: limbs < 1.5 2^30, < Y + 4r
        s1 = f29_reduce_qt(f29_lazy2(s1, u), qt);       // limbs < 2^31
        s2 = f29_reduce_qt(f29_lazy3(s2, s2, u), qt);   // limbs < 2.5 2^30
        x = r + 1 < rp ? f29_add(f29_lazy2(y, itl[r + 1]), u) : f29_add(y, u);  // < 2Y + 5r
    }
    return x;
}

// ---- pair-cooperative permutation, for levels of 16K..32K states: a quad per
// state would put two waves on a SIMD, one lane per state leaves half the SIMDs
// idle.  The even lane of a pair computes S-box 0, the odd lane S-box 1, both
// S-box 2; partial rounds as on a quad (x^4 and x^3 in parallel).  Critical
// path: 2 rf + rp S-boxes' worth of products (8 x 10 + 22 x 4 = 168 against
// 230 for one lane).  Both lanes of every pair must be active.
template <uint32_t D>
__device__ __forceinline__ F29 full_round_pair(F29& s0, F29& s1, F29& s2, const F29& t, const F29* __restrict__ c,
                                               uint32_t odd) {
    const uint32_t m1 = 0u - odd;
    F29 in;
#pragma unroll
    for (int i = 0; i < 9; ++i) in.l[i] = ((s0.l[i] + c[0].l[i]) & ~m1) | ((s1.l[i] + c[1].l[i]) & m1);
    const F29 xa = sbox29<D>(f29_add(in, t));
    s2 = sbox29<D>(f29_add(f29_lazy2(s2, c[2]), t));
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        s0.l[i] = pair_bcast(xa.l[i], 0);
        s1.l[i] = pair_bcast(xa.l[i], 1);
    }
    return f29_lazy3(s0, s1, s2);
}

template <uint32_t D>
__device__ __forceinline__ void permute3_f29_pair(F29& s0, F29& s1, F29& s2, const F29* __restrict__ rc29,
                                                  uint32_t rf, uint32_t rp, const uint4* __restrict__ qt) {
    const uint32_t odd = threadIdx.x & 1u;
    const uint32_t half = rf / 2;
    const F29* ini = rc29;
    const F29* ter = rc29 + 3 * half;
    const F29* itl = rc29 + 6 * half;
    F29 t = f29_lazy3(s0, s1, s2);
    for (uint32_t r = 0; r < half; ++r) t = full_round_pair<D>(s0, s1, s2, t, ini + 3 * r, odd);
    F29 x = rp ? f29_add(f29_lazy2(s0, itl[0]), t) : f29_add(s0, t);
    s1 = f29_reduce_qt(f29_lazy2(s1, t), qt);
    s2 = f29_reduce_qt(f29_lazy2(s2, t), qt);
    x = partial_rounds_f29<D, 2>(x, s1, s2, itl, rp, qt);
    s0 = x;
    t = f29_zero();
    for (uint32_t r = 0; r < half; ++r) t = full_round_pair<D>(s0, s1, s2, t, ter + 3 * r, odd);
    s0 = f29_add(s0, t);
    s1 = f29_add(s1, t);
    s2 = f29_add(s2, t);
}

template <uint32_t D>
__device__ __forceinline__ void permute3_f29_coop(F29& s0, F29& s1, F29& s2, const F29* __restrict__ rc29,
                                                  uint32_t rf, uint32_t rp, const uint4* __restrict__ qt) {
    const uint32_t j = min(threadIdx.x & 3u, 2u);
    const uint32_t half = rf / 2;
    const F29* ini = rc29;
    const F29* ter = rc29 + 3 * half;
    const F29* itl = rc29 + 6 * half;
    F29 t = f29_lazy3(s0, s1, s2);
    for (uint32_t r = 0; r < half; ++r) t = full_round_coop<D>(s0, s1, s2, t, ini + 3 * r, j);
    F29 x = rp ? f29_add(f29_lazy2(s0, itl[0]), t) : f29_add(s0, t);
    s1 = f29_reduce_qt(f29_lazy2(s1, t), qt);  // < 38.8 r, limbs < 2^31
    s2 = f29_reduce_qt(f29_lazy2(s2, t), qt);
    x = partial_rounds_f29<D, 4>(x, s1, s2, itl, rp, qt);
    s0 = x;
    t = f29_zero();
    for (uint32_t r = 0; r < half; ++r) t = full_round_coop<D>(s0, s1, s2, t, ter + 3 * r, j);
    s0 = f29_add(s0, t);
    s1 = f29_add(s1, t);
    s2 = f29_add(s2, t);
}

// ---- caller-set U2/U3 linear layers (lsp_params.internal_diag /
// external_mds; P2Layout::gen_lin).  The default layers above are additions
// folded lazily into the S-box inputs; a general M_E and M_I = J + diag(d)
// need products, so this variant keeps every state value normalised and
// < 2 r between layers (f29_reduce after each sum) and pays 9 products per
// external layer and 3 per internal layer.  Bounds: S-box inputs s + c < 4 r,
// outputs < 8.2 r; a layer's products (constants < 2 r) < 8.2 r, sums of
// three < 25 r < 2^261.  The constants follow the round constants in rc29:
// M_E row-major [9], then d [3] (poseidon2.hpp).  Kernels select it with the
// template flag P2_GEN on D.
constexpr uint32_t P2_GEN = 0x100u;

__device__ __forceinline__ void ext_layer_gen29(F29& s0, F29& s1, F29& s2, const F29* __restrict__ m) {
    F29 n[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        n[i] = f29_reduce(f29_add(f29_lazy2(f29_mul(m[3 * i], s0), f29_mul(m[3 * i + 1], s1)), f29_mul(m[3 * i + 2], s2)));
    s0 = n[0];
    s1 = n[1];
    s2 = n[2];
}

__device__ __forceinline__ void int_layer_gen29(F29& s0, F29& s1, F29& s2, const F29* __restrict__ d) {
    const F29 u = f29_lazy3(s0, s1, s2);  // < 12.2 r, limbs < 3 2^29
    s0 = f29_reduce(f29_add(u, f29_mul(d[0], s0)));
    s1 = f29_reduce(f29_add(u, f29_mul(d[1], s1)));
    s2 = f29_reduce(f29_add(u, f29_mul(d[2], s2)));
}

// the three S-boxes of a full round on 1, 2 (pair) or 4 (quad) lanes per state
template <uint32_t D, int LANES>
__device__ __forceinline__ void full_sboxes_gen29(F29& s0, F29& s1, F29& s2) {
    if constexpr (LANES == 1) {
        s0 = sbox29<D>(s0);
        s1 = sbox29<D>(s1);
        s2 = sbox29<D>(s2);
    } else if constexpr (LANES == 2) {
        const uint32_t m1 = 0u - (threadIdx.x & 1u);
        F29 in;
#pragma unroll
        for (int i = 0; i < 9; ++i) in.l[i] = (s0.l[i] & ~m1) | (s1.l[i] & m1);
        const F29 xa = sbox29<D>(in);
        s2 = sbox29<D>(s2);
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            s0.l[i] = pair_bcast(xa.l[i], 0);
            s1.l[i] = pair_bcast(xa.l[i], 1);
        }
    } else {
        const F29 x = sbox29<D>(f29_sel3(min(threadIdx.x & 3u, 2u), s0, s1, s2));
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            s0.l[i] = quad_bcast(x.l[i], 0);
            s1.l[i] = quad_bcast(x.l[i], 1);
            s2.l[i] = quad_bcast(x.l[i], 2);
        }
    }
}

template <uint32_t D, int LANES>
__device__ __forceinline__ void permute3_f29_gen(F29& s0, F29& s1, F29& s2, const F29* __restrict__ rc29,
                                                 uint32_t rf, uint32_t rp) {
    const uint32_t half = rf / 2;
    const F29* ini = rc29;
    const F29* ter = rc29 + 3 * half;
    const F29* itl = rc29 + 6 * half;
    const F29* lin = rc29 + 3 * rf + rp;
    ext_layer_gen29(s0, s1, s2, lin);
    for (uint32_t r = 0; r < half; ++r) {
        s0 = f29_add(s0, ini[3 * r + 0]);
        s1 = f29_add(s1, ini[3 * r + 1]);
        s2 = f29_add(s2, ini[3 * r + 2]);
        full_sboxes_gen29<D, LANES>(s0, s1, s2);
        ext_layer_gen29(s0, s1, s2, lin);
    }
    for (uint32_t r = 0; r < rp; ++r) {
        const F29 x = f29_add(s0, itl[r]);
        if constexpr (LANES == 1)
            s0 = sbox29<D>(x);
        else
            s0 = sbox29_coop<D, LANES>(x);
        int_layer_gen29(s0, s1, s2, lin + 9);
    }
    for (uint32_t r = 0; r < half; ++r) {
        s0 = f29_add(s0, ter[3 * r + 0]);
        s1 = f29_add(s1, ter[3 * r + 1]);
        s2 = f29_add(s2, ter[3 * r + 2]);
        full_sboxes_gen29<D, LANES>(s0, s1, s2);
        ext_layer_gen29(s0, s1, s2, lin);
    }
}

// LANES: lanes per state (1, 2: pair_, 4: quad-cooperative); D: the S-box
// degree, with P2_GEN set for caller-set linear layers
template <uint32_t D, int LANES = 1>
__device__ __forceinline__ void permute3_any(F29& s0, F29& s1, F29& s2, const F29* __restrict__ rc29, uint32_t rf,
                                             uint32_t rp, const uint4* __restrict__ qt) {
    if constexpr ((D & P2_GEN) != 0)
        permute3_f29_gen<(D & ~P2_GEN), LANES>(s0, s1, s2, rc29, rf, rp);
    else if (LANES == 4)
        permute3_f29_coop<D>(s0, s1, s2, rc29, rf, rp, qt);
    else if (LANES == 2)
        permute3_f29_pair<D>(s0, s1, s2, rc29, rf, rp, qt);
    else
        permute3_f29<D>(s0, s1, s2, rc29, rf, rp, qt);
}

// PaddingFreeSponge<Perm,3,2,1>::hash_iter over n elements read as ark-form Fr
// by get(k); returns the ark-form (canonical) digest
template <uint32_t D, int LANES = 1, class Get>
__device__ __forceinline__ Fr sponge_f29(Get get, uint32_t n, const F29* rc29, uint32_t rf, uint32_t rp,
                                         const uint4* __restrict__ qt) {
    F29 s0 = f29_zero(), s1 = f29_zero(), s2 = f29_zero();
    // the next block is loaded before the current permutation, so its memory
    // latency hides behind ~46 K instructions instead of stalling the wave
    Fr n0 = n > 0 ? get(0) : fr_zero(), n1 = n > 1 ? get(1) : fr_zero();
    uint32_t k = 0;
    while (k + 2 <= n) {
        s0 = f29_from_fr(n0);
        s1 = f29_from_fr(n1);
        if (k + 2 < n) n0 = get(k + 2);
        if (k + 3 < n) n1 = get(k + 3);
        permute3_any<D, LANES>(s0, s1, s2, rc29, rf, rp, qt);
        k += 2;
    }
    if (k < n) {
        s0 = f29_from_fr(n0);
        permute3_any<D, LANES>(s0, s1, s2, rc29, rf, rp, qt);
    }
    return f29_to_fr_qt(s0, qt);
}

template <uint32_t D, int LANES = 1>
__device__ __forceinline__ Fr compress_f29(const Fr& l, const Fr& r, const F29* rc29, uint32_t rf, uint32_t rp,
                                           const uint4* __restrict__ qt) {
    F29 s0 = f29_from_fr(l), s1 = f29_from_fr(r), s2 = f29_zero();
    permute3_any<D, LANES>(s0, s1, s2, rc29, rf, rp, qt);
    return f29_to_fr_qt(s0, qt);
}

}  // namespace lsp
