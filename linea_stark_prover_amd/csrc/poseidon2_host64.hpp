// Poseidon2Bls12337<3> on the host, in 4 x 64-bit limbs: the permutation the
// host runs on the critical path (Merkle tree tops, the challenger's sponge).
// Same function as permute3 (poseidon2.hpp, U1-U3 conventions) and the same
// in-memory element form (ark-ff Montgomery, R = 2^256: an Fr's eight 32-bit
// words are these four 64-bit limbs), but values stay lazily reduced in
// [0, 2r) between operations:
//   * product: CIOS without the final subtraction -- for inputs < 2r the
//     output is < 4r^2/2^256 + r < 1.3 r (r < 2^252.3);
//   * sum: a + b < 4r < 2^255, then one conditional subtraction of 2r;
//   * the permutation's outputs are made canonical ([0, r)) at the end.
#pragma once
#include <stdint.h>

#include "poseidon2.hpp"

namespace lsp {
namespace hp64 {

typedef unsigned __int128 u128;
struct F {
    uint64_t l[4];
};

// (host-only functions; the constants are spelled out so the header also
// parses in the device compilation pass)
constexpr uint64_t R0 = (uint64_t)LSP_MOD0 | ((uint64_t)LSP_MOD1 << 32), R1 = (uint64_t)LSP_MOD2 | ((uint64_t)LSP_MOD3 << 32),
                   R2 = (uint64_t)LSP_MOD4 | ((uint64_t)LSP_MOD5 << 32), R3 = (uint64_t)LSP_MOD6 | ((uint64_t)LSP_MOD7 << 32);
constexpr uint64_t inv64() {  // r^-1 mod 2^64 (Newton)
    uint64_t x = 1;
    for (int i = 0; i < 7; ++i) x *= 2 - R0 * x;
    return x;
}
constexpr uint64_t NP = 0 - inv64();  // -r^-1 mod 2^64
// 2r
constexpr uint64_t D0 = R0 << 1, D1 = (R1 << 1) | (R0 >> 63), D2 = (R2 << 1) | (R1 >> 63), D3 = (R3 << 1) | (R2 >> 63);

inline F from(const Fr& x) {
    F o;
    __builtin_memcpy(o.l, x.v, 32);
    return o;
}

// a - m if a >= m, else a (m = the 4-limb constant)
inline F csub(const F& a, uint64_t m0, uint64_t m1, uint64_t m2, uint64_t m3) {
    uint64_t d[4];
    u128 v = (u128)a.l[0] - m0;
    d[0] = (uint64_t)v;
    v = (u128)a.l[1] - m1 - (uint64_t)((v >> 64) & 1);
    d[1] = (uint64_t)v;
    v = (u128)a.l[2] - m2 - (uint64_t)((v >> 64) & 1);
    d[2] = (uint64_t)v;
    v = (u128)a.l[3] - m3 - (uint64_t)((v >> 64) & 1);
    d[3] = (uint64_t)v;
    const uint64_t keep = 0 - (uint64_t)((v >> 64) & 1);  // borrow: a < m
    F o;
    for (int i = 0; i < 4; ++i) o.l[i] = (a.l[i] & keep) | (d[i] & ~keep);
    return o;
}

inline Fr to_canonical(const F& x) {
    const F c = csub(x, R0, R1, R2, R3);
    Fr o;
    __builtin_memcpy(o.v, c.l, 32);
    return o;
}

inline F add(const F& a, const F& b) {
    F s;
    u128 c = (u128)a.l[0] + b.l[0];
    s.l[0] = (uint64_t)c;
    c = (u128)a.l[1] + b.l[1] + (uint64_t)(c >> 64);
    s.l[1] = (uint64_t)c;
    c = (u128)a.l[2] + b.l[2] + (uint64_t)(c >> 64);
    s.l[2] = (uint64_t)c;
    s.l[3] = a.l[3] + b.l[3] + (uint64_t)(c >> 64);
    return csub(s, D0, D1, D2, D3);
}

// a - b as a + (2r - b), for b < 2r: < 4r, then one conditional subtraction of 2r
inline F sub(const F& a, const F& b) {
    F n;
    u128 c = (u128)D0 - b.l[0];
    n.l[0] = (uint64_t)c;
    c = (u128)D1 - b.l[1] - (uint64_t)((c >> 64) & 1);
    n.l[1] = (uint64_t)c;
    c = (u128)D2 - b.l[2] - (uint64_t)((c >> 64) & 1);
    n.l[2] = (uint64_t)c;
    n.l[3] = D3 - b.l[3] - (uint64_t)((c >> 64) & 1);
    return add(a, n);
}

inline F mul_u128(const F& a, const F& b) {
    uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    for (int i = 0; i < 4; ++i) {
        const uint64_t y = b.l[i];
        u128 c = (u128)a.l[0] * y + t0;
        t0 = (uint64_t)c;
        c = (u128)a.l[1] * y + t1 + (uint64_t)(c >> 64);
        t1 = (uint64_t)c;
        c = (u128)a.l[2] * y + t2 + (uint64_t)(c >> 64);
        t2 = (uint64_t)c;
        c = (u128)a.l[3] * y + t3 + (uint64_t)(c >> 64);
        t3 = (uint64_t)c;
        t4 += (uint64_t)(c >> 64);
        const uint64_t m = t0 * NP;
        c = (u128)m * R0 + t0;
        c = (u128)m * R1 + t1 + (uint64_t)(c >> 64);
        t0 = (uint64_t)c;
        c = (u128)m * R2 + t2 + (uint64_t)(c >> 64);
        t1 = (uint64_t)c;
        c = (u128)m * R3 + t3 + (uint64_t)(c >> 64);
        t2 = (uint64_t)c;
        c = (u128)t4 + (uint64_t)(c >> 64);
        t3 = (uint64_t)c;
        t4 = (uint64_t)(c >> 64);
    }
    return F{{t0, t1, t2, t3}};
}


// x R^-1 (Montgomery form -> the integer), i.e. mul(x, 1) without the
// products by b's limbs: four reduction rows of one imul + 4 multiplies.
// Input < 2r (any value < 2^256 works: the result is < r + 1), output < 2r.
inline F redc(const F& a) {
    uint64_t t0 = a.l[0], t1 = a.l[1], t2 = a.l[2], t3 = a.l[3];
    for (int i = 0; i < 4; ++i) {
        const uint64_t m = t0 * NP;
        u128 c = (u128)m * R0 + t0;
        c = (u128)m * R1 + t1 + (uint64_t)(c >> 64);
        t0 = (uint64_t)c;
        c = (u128)m * R2 + t2 + (uint64_t)(c >> 64);
        t1 = (uint64_t)c;
        c = (u128)m * R3 + t3 + (uint64_t)(c >> 64);
        t2 = (uint64_t)c;
        t3 = (uint64_t)(c >> 64);
    }
    return F{{t0, t1, t2, t3}};
}

#if defined(__x86_64__) && defined(__ADX__) && defined(__BMI2__) && !defined(__HIP_DEVICE_COMPILE__)
// The same CIOS (same digits m, same result bits) with mulx and the two carry
// chains adcx / adox: ~30 % less latency than the compiler's code for
// mul_u128, which matters for the host's sequential permutations (transcript
// samples, the narrowest tree-top levels).  Inputs < 2r keep every row's
// accumulator below 2^318, so no carry leaves the top limb.
inline F mul(const F& a, const F& b) {
    static const uint64_t K[5] = {R0, R1, R2, R3, NP};
    uint64_t t0, t1, t2, t3, t4, lo, hi, zero = 0;
    __asm__(
        "movq 0(%[b]), %%rdx\n\t"
        "xorl %k[t4], %k[t4]\n\t"
        "mulxq 0(%[a]), %[t0], %[t1]\n\t"
        "mulxq 8(%[a]), %[lo], %[t2]\n\t"
        "adcxq %[lo], %[t1]\n\t"
        "mulxq 16(%[a]), %[lo], %[t3]\n\t"
        "adcxq %[lo], %[t2]\n\t"
        "mulxq 24(%[a]), %[lo], %[hi]\n\t"
        "adcxq %[lo], %[t3]\n\t"
        "adcxq %[hi], %[t4]\n\t"
        "movq %[t0], %%rdx\n\t"
        "imulq 32(%[k]), %%rdx\n\t"
        "xorl %k[zero], %k[zero]\n\t"
        "mulxq 0(%[k]), %[lo], %[hi]\n\t"
        "adoxq %[lo], %[t0]\n\t"
        "adcxq %[hi], %[t1]\n\t"
        "mulxq 8(%[k]), %[lo], %[hi]\n\t"
        "adoxq %[lo], %[t1]\n\t"
        "adcxq %[hi], %[t2]\n\t"
        "mulxq 16(%[k]), %[lo], %[hi]\n\t"
        "adoxq %[lo], %[t2]\n\t"
        "adcxq %[hi], %[t3]\n\t"
        "mulxq 24(%[k]), %[lo], %[hi]\n\t"
        "adoxq %[lo], %[t3]\n\t"
        "adcxq %[hi], %[t4]\n\t"
        "adoxq %[zero], %[t4]\n\t"
        : [t0] "=&r"(t0), [t1] "=&r"(t1), [t2] "=&r"(t2), [t3] "=&r"(t3), [t4] "=&r"(t4), [lo] "=&r"(lo),
          [hi] "=&r"(hi), [zero] "+&r"(zero)
        : [a] "r"(a.l), [b] "r"(b.l), [k] "r"(K)
        : "rdx", "cc", "memory");
    for (int i = 1; i < 4; ++i) {
        uint64_t t5;
        __asm__(
            "movq (%[bi]), %%rdx\n\t"
            "xorl %k[t5], %k[t5]\n\t"
            "mulxq 0(%[a]), %[lo], %[hi]\n\t"
            "adoxq %[lo], %[t1]\n\t"
            "adcxq %[hi], %[t2]\n\t"
            "mulxq 8(%[a]), %[lo], %[hi]\n\t"
            "adoxq %[lo], %[t2]\n\t"
            "adcxq %[hi], %[t3]\n\t"
            "mulxq 16(%[a]), %[lo], %[hi]\n\t"
            "adoxq %[lo], %[t3]\n\t"
            "adcxq %[hi], %[t4]\n\t"
            "mulxq 24(%[a]), %[lo], %[hi]\n\t"
            "adoxq %[lo], %[t4]\n\t"
            "adcxq %[hi], %[t5]\n\t"
            "movl $0, %k[lo]\n\t"
            "adoxq %[lo], %[t5]\n\t"
            "movq %[t1], %%rdx\n\t"
            "imulq 32(%[k]), %%rdx\n\t"
            "xorl %k[lo], %k[lo]\n\t"
            "mulxq 0(%[k]), %[lo], %[hi]\n\t"
            "adoxq %[lo], %[t1]\n\t"
            "adcxq %[hi], %[t2]\n\t"
            "mulxq 8(%[k]), %[lo], %[hi]\n\t"
            "adoxq %[lo], %[t2]\n\t"
            "adcxq %[hi], %[t3]\n\t"
            "mulxq 16(%[k]), %[lo], %[hi]\n\t"
            "adoxq %[lo], %[t3]\n\t"
            "adcxq %[hi], %[t4]\n\t"
            "mulxq 24(%[k]), %[lo], %[hi]\n\t"
            "adoxq %[lo], %[t4]\n\t"
            "adcxq %[hi], %[t5]\n\t"
            "movl $0, %k[lo]\n\t"
            "adoxq %[lo], %[t5]\n\t"
            : [t1] "+&r"(t1), [t2] "+&r"(t2), [t3] "+&r"(t3), [t4] "+&r"(t4), [t5] "=&r"(t5), [lo] "=&r"(lo),
              [hi] "=&r"(hi)
            : [a] "r"(a.l), [bi] "r"(b.l + i), [k] "r"(K)
            : "rdx", "cc", "memory");
        t1 = t2;
        t2 = t3;
        t3 = t4;
        t4 = t5;
    }
    return F{{t1, t2, t3, t4}};
}
#else
inline F mul(const F& a, const F& b) { return mul_u128(a, b); }
#endif

// x^11 = (x^4)^2 x^3 with x^3 and x^4 independent: a chain of 4 products
// instead of 5 (the core runs the two middle ones side by side) -- the host's
// permutations are latency-bound (tree tops, transcript samples)
template <uint32_t D>
inline F sbox(const F& x) {
    const F x2 = mul(x, x);
#ifndef LSP_HOST_SBOX5  // A/B switch: the 5-product chain x^8 x^2 x
    if (D == 11) {
        const F x3 = mul(x2, x);
        const F x4 = mul(x2, x2);
        return mul(mul(x4, x4), x3);
    }
#endif
    const F x4 = mul(x2, x2);
    const F x8 = mul(x4, x4);
    if (D == 11) return mul(mul(x8, x2), x);
    return mul(mul(x8, x8), x);  // x^17
}

inline void ext_layer(F& s0, F& s1, F& s2) {
    const F t = add(add(s0, s1), s2);
    s0 = add(s0, t);
    s1 = add(s1, t);
    s2 = add(s2, t);
}

// caller-set U2/U3 layers (P2Layout::gen_lin): s <- M_E s and
// s_i <- (s0 + s1 + s2) + d_i s_i, products of values < 2r (< 1.3 r)
inline void ext_layer_gen(F& s0, F& s1, F& s2, const Fr* m) {
    F n[3];
    for (int i = 0; i < 3; ++i)
        n[i] = add(add(mul(from(m[3 * i]), s0), mul(from(m[3 * i + 1]), s1)), mul(from(m[3 * i + 2]), s2));
    s0 = n[0];
    s1 = n[1];
    s2 = n[2];
}

inline void int_layer_gen(F& s0, F& s1, F& s2, const Fr* d) {
    const F t = add(add(s0, s1), s2);
    s0 = add(t, mul(from(d[0]), s0));
    s1 = add(t, mul(from(d[1]), s1));
    s2 = add(t, mul(from(d[2]), s2));
}

// rc: constants in new_from_rng order (poseidon2.hpp); states in and out
// canonical.  lin: nullptr = the default U2/U3 layers, else M_E [9] then d [3]
template <uint32_t D>
inline void permute3(Fr& a0, Fr& a1, Fr& a2, const Fr* rc, uint32_t rounds_f, uint32_t rounds_p,
                     const Fr* lin = nullptr) {
    const uint32_t half = rounds_f / 2;
    const Fr* ini = rc;
    const Fr* ter = rc + 3 * half;
    const Fr* itl = rc + 6 * half;
    F s0 = from(a0), s1 = from(a1), s2 = from(a2);
    auto ext = [&] {
        if (lin)
            ext_layer_gen(s0, s1, s2, lin);
        else
            ext_layer(s0, s1, s2);
    };
    ext();
    for (uint32_t r = 0; r < half; ++r) {
        s0 = sbox<D>(add(s0, from(ini[3 * r + 0])));
        s1 = sbox<D>(add(s1, from(ini[3 * r + 1])));
        s2 = sbox<D>(add(s2, from(ini[3 * r + 2])));
        ext();
    }
    for (uint32_t r = 0; r < rounds_p; ++r) {
        s0 = sbox<D>(add(s0, from(itl[r])));
        if (lin) {
            int_layer_gen(s0, s1, s2, lin + 9);
            continue;
        }
        const F t = add(add(s0, s1), s2);
        s0 = add(s0, t);
        s1 = add(s1, t);
        s2 = add(add(s2, s2), t);
    }
    for (uint32_t r = 0; r < half; ++r) {
        s0 = sbox<D>(add(s0, from(ter[3 * r + 0])));
        s1 = sbox<D>(add(s1, from(ter[3 * r + 1])));
        s2 = sbox<D>(add(s2, from(ter[3 * r + 2])));
        ext();
    }
    a0 = to_canonical(s0);
    a1 = to_canonical(s1);
    a2 = to_canonical(s2);
}

inline void permute3_rt(Fr& s0, Fr& s1, Fr& s2, const Fr* rc, const P2Layout& L) {
    const Fr* lin = L.gen_lin ? rc + p2_lin_offset(L) : nullptr;
    if (L.sbox_degree == 17)
        permute3<17>(s0, s1, s2, rc, L.rounds_f, L.rounds_p, lin);
    else
        permute3<11>(s0, s1, s2, rc, L.rounds_f, L.rounds_p, lin);
}

}  // namespace hp64
}  // namespace lsp
