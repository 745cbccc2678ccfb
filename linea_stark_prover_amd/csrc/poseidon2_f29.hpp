// Poseidon2Bls12337<3> on the 29-bit-limb representation (fr29.hpp).
// Same permutation as poseidon2.hpp (U1-U3 conventions); only the arithmetic
// representation differs.  Lazy-reduction bounds (r = the field modulus):
//   S-box inputs < 32 r (f29_mul requirement), outputs < 3.3 r;
//   full rounds: state < 5.5 r after the external layer;
//   partial rounds: t = reduce(s0 + s1 + s2) < 2 r, s2 reduced every round
//   (it doubles), s1 grows by < 2 r per round and is reduced once after the
//   partial rounds (< 50 r < 2^259 in between).
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

__device__ __forceinline__ void ext_layer29(F29& s0, F29& s1, F29& s2) {
    const F29 t = f29_add(f29_add(s0, s1), s2);
    s0 = f29_add(s0, t);
    s1 = f29_add(s1, t);
    s2 = f29_add(s2, t);
}

// rc29: round constants in F29 form, new_from_rng order (initial external
// [rf/2][3], terminal external [rf/2][3], internal [rp])
template <uint32_t D>
__device__ __forceinline__ void permute3_f29(F29& s0, F29& s1, F29& s2, const F29* __restrict__ rc29, uint32_t rf,
                                             uint32_t rp) {
    const uint32_t half = rf / 2;
    const F29* ini = rc29;
    const F29* ter = rc29 + 3 * half;
    const F29* itl = rc29 + 6 * half;
    ext_layer29(s0, s1, s2);
    for (uint32_t r = 0; r < half; ++r) {
        s0 = sbox29<D>(f29_add(s0, ini[3 * r + 0]));
        s1 = sbox29<D>(f29_add(s1, ini[3 * r + 1]));
        s2 = sbox29<D>(f29_add(s2, ini[3 * r + 2]));
        ext_layer29(s0, s1, s2);
    }
    s1 = f29_reduce(s1);
    s2 = f29_reduce(s2);
    for (uint32_t r = 0; r < rp; ++r) {
        s0 = sbox29<D>(f29_add(s0, itl[r]));
        const F29 t = f29_reduce(f29_add(f29_add(s0, s1), s2));
        s0 = f29_add(s0, t);
        s1 = f29_add(s1, t);
        s2 = f29_reduce(f29_add(f29_add(s2, s2), t));
    }
    s1 = f29_reduce(s1);
    for (uint32_t r = 0; r < half; ++r) {
        s0 = sbox29<D>(f29_add(s0, ter[3 * r + 0]));
        s1 = sbox29<D>(f29_add(s1, ter[3 * r + 1]));
        s2 = sbox29<D>(f29_add(s2, ter[3 * r + 2]));
        ext_layer29(s0, s1, s2);
    }
}

__device__ __forceinline__ F29 f29_zero() {
    F29 z;
#pragma unroll
    for (int i = 0; i < 9; ++i) z.l[i] = 0;
    return z;
}

// PaddingFreeSponge<Perm,3,2,1>::hash_iter over n elements read as ark-form Fr
// by get(k); returns the ark-form (canonical) digest
template <uint32_t D, class Get>
__device__ __forceinline__ Fr sponge_f29(Get get, uint32_t n, const F29* rc29, uint32_t rf, uint32_t rp) {
    F29 s0 = f29_zero(), s1 = f29_zero(), s2 = f29_zero();
    uint32_t k = 0;
    while (k + 2 <= n) {
        s0 = f29_from_fr(get(k));
        s1 = f29_from_fr(get(k + 1));
        permute3_f29<D>(s0, s1, s2, rc29, rf, rp);
        k += 2;
    }
    if (k < n) {
        s0 = f29_from_fr(get(k));
        permute3_f29<D>(s0, s1, s2, rc29, rf, rp);
    }
    return f29_to_fr(s0);
}

template <uint32_t D>
__device__ __forceinline__ Fr compress_f29(const Fr& l, const Fr& r, const F29* rc29, uint32_t rf, uint32_t rp) {
    F29 s0 = f29_from_fr(l), s1 = f29_from_fr(r), s2 = f29_zero();
    permute3_f29<D>(s0, s1, s2, rc29, rf, rp);
    return f29_to_fr(s0);
}

}  // namespace lsp
