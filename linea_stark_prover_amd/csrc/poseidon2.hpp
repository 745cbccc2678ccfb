// Poseidon2Bls12337<3> (bin/src/config.rs:11; Perm::new_from_rng(8, 22),
// bin/src/main.rs:49) and the sponge / compression built on it
// (PaddingFreeSponge<Perm,3,2,1>, bin/src/config.rs:12;
// CompressionFunctionFromHasher<Hash,2,1>, bin/src/config.rs:17).
//
// Conventions (parity unpinned): U1 S-box x^d (d = 11 default,
// 17 allowed); U2 internal layer s_i += sum with s2 doubled first
// (diag (1,1,2)); U3 external layer circ(2,1,1) = s_i += sum, applied once
// before the first full round.  Round constants (U4) are supplied by the
// caller in new_from_rng order: initial external [rf/2][3], terminal external
// [rf/2][3], internal [rp].  The 8 x 32-bit permute3 below has the default
// U2/U3 layers only (micro-benchmarks); the product's permutations
// (poseidon2_f29.hpp, poseidon2_host64.hpp, host_ifma.cpp) also take
// caller-set layers (P2Layout::gen_lin).
#pragma once
#include "fr.hpp"

namespace lsp {

// gen_lin: non-default U2/U3 linear layers (lsp_params.internal_diag /
// external_mds).  Their constants follow the round constants in every
// constant array (host Fr, device F29, IFMA lanes): M_E row-major [9], then
// the internal diagonal d [3] (p2_lin_offset).
struct P2Layout {
    uint32_t rounds_f, rounds_p, sbox_degree;
    uint32_t gen_lin = 0;
};
constexpr uint32_t P2_LIN_N = 12;
LSP_HD uint32_t p2_lin_offset(const P2Layout& L) { return 3 * L.rounds_f + L.rounds_p; }

LSP_HD Fr sbox(const Fr& x, uint32_t d) {
    Fr x2 = fr_sqr(x);
    Fr x4 = fr_sqr(x2);
    Fr x8 = fr_sqr(x4);
    if (d == 11) {
        return fr_mul(fr_mul(x8, x2), x);  // x^11 = x^8 x^2 x
    }
    // d == 17: x^16 x
    return fr_mul(fr_sqr(x8), x);
}

LSP_HD void ext_layer(Fr& s0, Fr& s1, Fr& s2) {
    Fr t = fr_add(fr_add(s0, s1), s2);
    s0 = fr_add(s0, t);
    s1 = fr_add(s1, t);
    s2 = fr_add(s2, t);
}

LSP_HD void int_layer(Fr& s0, Fr& s1, Fr& s2) {
    Fr t = fr_add(fr_add(s0, s1), s2);
    s0 = fr_add(s0, t);
    s1 = fr_add(s1, t);
    s2 = fr_add(fr_dbl(s2), t);
}

// rc: constants in new_from_rng order (see header comment)
template <uint32_t D>
LSP_HD void permute3(Fr& s0, Fr& s1, Fr& s2, const Fr* __restrict__ rc, uint32_t rounds_f,
                     uint32_t rounds_p) {
    const uint32_t half = rounds_f / 2;
    const Fr* ini = rc;
    const Fr* ter = rc + 3 * half;
    const Fr* itl = rc + 6 * half;
    ext_layer(s0, s1, s2);
    for (uint32_t r = 0; r < half; ++r) {
        s0 = sbox(fr_add(s0, ini[3 * r + 0]), D);
        s1 = sbox(fr_add(s1, ini[3 * r + 1]), D);
        s2 = sbox(fr_add(s2, ini[3 * r + 2]), D);
        ext_layer(s0, s1, s2);
    }
    for (uint32_t r = 0; r < rounds_p; ++r) {
        s0 = sbox(fr_add(s0, itl[r]), D);
        int_layer(s0, s1, s2);
    }
    for (uint32_t r = 0; r < half; ++r) {
        s0 = sbox(fr_add(s0, ter[3 * r + 0]), D);
        s1 = sbox(fr_add(s1, ter[3 * r + 1]), D);
        s2 = sbox(fr_add(s2, ter[3 * r + 2]), D);
        ext_layer(s0, s1, s2);
    }
}

// PaddingFreeSponge<Perm,3,2,1>::hash_iter over n elements read by `get(k)`:
// overwrite-mode absorb of 2 per permutation; a partial last block overwrites
// only lane 0 and still permutes; an exact multiple of 2 ends without an extra
// permutation; output lane 0.
template <uint32_t D, class Get>
LSP_HD Fr sponge(Get get, uint32_t n, const Fr* rc, uint32_t rounds_f, uint32_t rounds_p) {
    Fr s0 = fr_zero(), s1 = fr_zero(), s2 = fr_zero();
    uint32_t k = 0;
    while (k + 2 <= n) {
        s0 = get(k);
        s1 = get(k + 1);
        permute3<D>(s0, s1, s2, rc, rounds_f, rounds_p);
        k += 2;
    }
    if (k < n) {
        s0 = get(k);
        permute3<D>(s0, s1, s2, rc, rounds_f, rounds_p);
    }
    return s0;
}

template <uint32_t D>
LSP_HD Fr compress2(const Fr& l, const Fr& r, const Fr* rc, uint32_t rounds_f, uint32_t rounds_p) {
    Fr s0 = l, s1 = r, s2 = fr_zero();
    permute3<D>(s0, s1, s2, rc, rounds_f, rounds_p);
    return s0;
}

}  // namespace lsp
