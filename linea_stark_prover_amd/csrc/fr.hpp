// BLS12-377 scalar field Fr for CDNA4 (gfx950) and the host.
//
// Replaces ark-ff 0.5's Montgomery Fr (Cargo.lock:83) as reached through
// p3-bls12-377-fr (bin/src/config.rs:1,9-10).  Same in-memory form as ark-ff:
// Montgomery with R = 2^256, little-endian limbs, canonical in [0, r) at every
// boundary -- here as 8 x 32-bit limbs, which is what the VALU multiplies
// (v_mad_u64_u32: 32x32+64 -> 64).
//
// Montgomery product: CIOS, 32-bit words, "no-carry" variant (valid because
// r's top word 0x12ab655e < 2^31 - 1).  r = 1 mod 2^47 gives r[0] = 1 and
// -r^-1 mod 2^32 = 0xffffffff, so the per-word quotient digit is m = -t0 and
// the m*r[0] term collapses to a carry of (t0 != 0).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LSP_HD __host__ __device__ __forceinline__

namespace lsp {

struct alignas(16) Fr {
    uint32_t v[8];
};

// r, little-endian 32-bit words
#define LSP_MOD0 0x00000001u
#define LSP_MOD1 0x0a118000u
#define LSP_MOD2 0xd0000001u
#define LSP_MOD3 0x59aa76feu
#define LSP_MOD4 0x5c37b001u
#define LSP_MOD5 0x60b44d1eu
#define LSP_MOD6 0x9a2ca556u
#define LSP_MOD7 0x12ab655eu

LSP_HD uint32_t mod_word(int i) {
    switch (i) {
        case 0: return LSP_MOD0;
        case 1: return LSP_MOD1;
        case 2: return LSP_MOD2;
        case 3: return LSP_MOD3;
        case 4: return LSP_MOD4;
        case 5: return LSP_MOD5;
        case 6: return LSP_MOD6;
        default: return LSP_MOD7;
    }
}

LSP_HD Fr fr_zero() {
    Fr r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = 0;
    return r;
}

// Montgomery one = 2^256 mod r
LSP_HD Fr fr_one() {
    Fr r;
    r.v[0] = 0xfffffff3u; r.v[1] = 0x7d1c7fffu; r.v[2] = 0x6ffffff2u; r.v[3] = 0x7257f50fu;
    r.v[4] = 0x512c0feeu; r.v[5] = 0x16d81575u; r.v[6] = 0x2bbb9a9du; r.v[7] = 0x0d4bda32u;
    return r;
}

// R^2 mod r (to enter Montgomery form)
LSP_HD Fr fr_r2() {
    Fr r;
    r.v[0] = 0xb861857bu; r.v[1] = 0x25d577bau; r.v[2] = 0x8860591fu; r.v[3] = 0xcc2c27b5u;
    r.v[4] = 0xe5dc8593u; r.v[5] = 0xa7cc008fu; r.v[6] = 0xeff1c939u; r.v[7] = 0x011fdae7u;
    return r;
}

LSP_HD bool fr_eq(const Fr& a, const Fr& b) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d |= a.v[i] ^ b.v[i];
    return d == 0;
}

LSP_HD bool fr_is_zero(const Fr& a) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d |= a.v[i];
    return d == 0;
}

// x - r if x >= r else x, for x < 2r
LSP_HD Fr fr_reduce_once(const Fr& x) {
    Fr d;
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t t = (uint64_t)x.v[i] - mod_word(i) - borrow;
        d.v[i] = (uint32_t)t;
        borrow = (uint32_t)(t >> 63);
    }
    Fr r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = borrow ? x.v[i] : d.v[i];
    return r;
}

LSP_HD Fr fr_add(const Fr& a, const Fr& b) {
    Fr s;
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t t = (uint64_t)a.v[i] + b.v[i] + c;
        s.v[i] = (uint32_t)t;
        c = t >> 32;
    }
    return fr_reduce_once(s);
}

LSP_HD Fr fr_sub(const Fr& a, const Fr& b) {
    Fr d;
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t t = (uint64_t)a.v[i] - b.v[i] - borrow;
        d.v[i] = (uint32_t)t;
        borrow = (uint32_t)(t >> 63);
    }
    // add r back when the subtraction wrapped
    uint32_t mask = 0u - borrow;
    Fr r;
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t t = (uint64_t)d.v[i] + (mod_word(i) & mask) + c;
        r.v[i] = (uint32_t)t;
        c = t >> 32;
    }
    return r;
}

LSP_HD Fr fr_neg(const Fr& a) { return fr_sub(fr_zero(), a); }
LSP_HD Fr fr_dbl(const Fr& a) { return fr_add(a, a); }

// Portable CIOS (host, and the reference point of the device multiplier)
LSP_HD Fr fr_mul_cios(const Fr& a, const Fr& b) {
    uint32_t t[8];
    // i = 0 (t = 0)
    {
        const uint32_t bi = b.v[0];
        uint64_t p = (uint64_t)a.v[0] * bi;
        uint32_t A = (uint32_t)(p >> 32);
        uint32_t t0 = (uint32_t)p;
        uint32_t m = 0u - t0;
        uint32_t C = t0 != 0u;
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            p = (uint64_t)a.v[j] * bi + A;
            A = (uint32_t)(p >> 32);
            uint32_t tj = (uint32_t)p;
            p = (uint64_t)m * mod_word(j) + tj + C;
            C = (uint32_t)(p >> 32);
            t[j - 1] = (uint32_t)p;
        }
        t[7] = C + A;
    }
#pragma unroll
    for (int i = 1; i < 8; ++i) {
        const uint32_t bi = b.v[i];
        uint64_t p = (uint64_t)a.v[0] * bi + t[0];
        uint32_t A = (uint32_t)(p >> 32);
        uint32_t t0 = (uint32_t)p;
        uint32_t m = 0u - t0;
        uint32_t C = t0 != 0u;
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            p = (uint64_t)a.v[j] * bi + t[j] + A;
            A = (uint32_t)(p >> 32);
            uint32_t tj = (uint32_t)p;
            p = (uint64_t)m * mod_word(j) + tj + C;
            C = (uint32_t)(p >> 32);
            t[j - 1] = (uint32_t)p;
        }
        t[7] = C + A;
    }
    Fr r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = t[i];
    return fr_reduce_once(r);
}

#if defined(__HIP_DEVICE_COMPILE__)
// gfx950 device product: FIPS with one inline-asm block per column
// (generated by tools/gen_frmul.py)
#include "fr_mul_gfx950.inc"
#endif

#if !defined(__HIP_DEVICE_COMPILE__)
// Host product: CIOS on 4 x 64-bit words with 128-bit products (the same
// Montgomery domain, R = 2^256, so bit-identical to the device product).  It
// serves the transcript, the verifier and the Merkle tree tops the prover
// finishes on the host.
namespace host64 {
constexpr uint64_t P0 = (uint64_t)LSP_MOD0 | ((uint64_t)LSP_MOD1 << 32);
constexpr uint64_t P1 = (uint64_t)LSP_MOD2 | ((uint64_t)LSP_MOD3 << 32);
constexpr uint64_t P2 = (uint64_t)LSP_MOD4 | ((uint64_t)LSP_MOD5 << 32);
constexpr uint64_t P3 = (uint64_t)LSP_MOD6 | ((uint64_t)LSP_MOD7 << 32);
constexpr uint64_t inv64() {  // r^-1 mod 2^64 (Newton: each step doubles the correct bits)
    uint64_t x = 1;
    for (int i = 0; i < 7; ++i) x *= 2 - P0 * x;
    return x;
}
constexpr uint64_t NP = 0 - inv64();  // -r^-1 mod 2^64
}  // namespace host64

inline Fr fr_mul_host64(const Fr& a, const Fr& b) {
    using namespace host64;
    typedef unsigned __int128 u128;
    static const uint64_t P[4] = {P0, P1, P2, P3};
    uint64_t x[4], y[4];
    __builtin_memcpy(x, a.v, 32);
    __builtin_memcpy(y, b.v, 32);
    uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    for (int i = 0; i < 4; ++i) {
        u128 c = (u128)x[0] * y[i] + t0;
        t0 = (uint64_t)c;
        c = (u128)x[1] * y[i] + t1 + (uint64_t)(c >> 64);
        t1 = (uint64_t)c;
        c = (u128)x[2] * y[i] + t2 + (uint64_t)(c >> 64);
        t2 = (uint64_t)c;
        c = (u128)x[3] * y[i] + t3 + (uint64_t)(c >> 64);
        t3 = (uint64_t)c;
        t4 += (uint64_t)(c >> 64);  // t4 stays tiny: inputs < r < 2^253
        const uint64_t m = t0 * NP;
        c = (u128)m * P[0] + t0;
        c = (u128)m * P[1] + t1 + (uint64_t)(c >> 64);
        t0 = (uint64_t)c;
        c = (u128)m * P[2] + t2 + (uint64_t)(c >> 64);
        t1 = (uint64_t)c;
        c = (u128)m * P[3] + t3 + (uint64_t)(c >> 64);
        t2 = (uint64_t)c;
        c = (u128)t4 + (uint64_t)(c >> 64);
        t3 = (uint64_t)c;
        t4 = (uint64_t)(c >> 64);
    }
    uint64_t r[4] = {t0, t1, t2, t3};
    // result < 2r: subtract r once if r[] >= P
    uint64_t d[4];
    u128 bw = 0;
    for (int k = 0; k < 4; ++k) {
        const u128 v = (u128)r[k] - P[k] - (uint64_t)bw;
        d[k] = (uint64_t)v;
        bw = (v >> 64) & 1;
    }
    Fr out;
    __builtin_memcpy(out.v, (t4 || !bw) ? d : r, 32);
    return out;
}
#endif

LSP_HD Fr fr_mul(const Fr& a, const Fr& b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return fr_mul_dev(a, b);
#else
    return fr_mul_host64(a, b);
#endif
}

LSP_HD Fr fr_sqr(const Fr& a) { return fr_mul(a, a); }

// a^e for a 64-bit exponent (left-to-right)
LSP_HD Fr fr_pow_u64(const Fr& a, uint64_t e) {
    Fr r = fr_one();
    bool started = false;
    for (int k = 63; k >= 0; --k) {
        if (started) r = fr_sqr(r);
        if ((e >> k) & 1u) {
            r = started ? fr_mul(r, a) : a;
            started = true;
        }
    }
    return r;
}

// a^(r-2) (Fermat); inverse of zero is zero
LSP_HD Fr fr_inv(const Fr& a) {
    Fr r = fr_one();
    bool started = false;
    for (int w = 7; w >= 0; --w) {
        // r - 2: r[0] = 1, so the subtraction borrows from word 1
        uint32_t e = w == 0 ? 0xffffffffu : (w == 1 ? LSP_MOD1 - 1u : mod_word(w));
        for (int k = 31; k >= 0; --k) {
            if (started) r = fr_sqr(r);
            if ((e >> k) & 1u) {
                r = started ? fr_mul(r, a) : a;
                started = true;
            }
        }
    }
    return r;
}

// integer -> Montgomery form
LSP_HD Fr fr_from_u64(uint64_t x) {
    Fr c = fr_zero();
    c.v[0] = (uint32_t)x;
    c.v[1] = (uint32_t)(x >> 32);
    return fr_mul(c, fr_r2());
}

// Montgomery -> canonical integer words
LSP_HD Fr fr_to_canonical(const Fr& a) {
    Fr one = fr_zero();
    one.v[0] = 1;
    return fr_mul(a, one);
}

LSP_HD Fr fr_from_canonical(const Fr& c) { return fr_mul(c, fr_r2()); }

// canonical words < r ?
LSP_HD bool fr_words_lt_mod(const Fr& c) {
    for (int i = 7; i >= 0; --i) {
        if (c.v[i] < mod_word(i)) return true;
        if (c.v[i] > mod_word(i)) return false;
    }
    return false;
}

}  // namespace lsp
