// Fr in 9 x 29-bit limbs on gfx950: the Poseidon2 working representation.
//
// Why: with 29-bit limbs every 29x29-bit product is < 2^58, so a whole
// FIPS column (at most 9 + 8 products plus the carry) fits in one 64-bit
// accumulator: each product is a single v_mad_u64_u32 with no carry-out to
// fold (the 32-bit-limb FIPS needs a v_addc_co_u32 after every product).
// 153 mads per product instead of 121 mads + 120 adds.
//
// Representation: x is held as X = x * 2^261 mod r ("Montgomery, R' = 2^261")
// in limbs l[0..8] of 29 bits (l[8] may hold a few more bits).  Values are
// kept lazily reduced; the invariants (see f29_mul_c) are
//   mul inputs  < K r (< 2^261) with normalised limbs (limbs 0..7 < 2^29)
//   ->  mul output normalised and < (8 + 0.0023 K^2) r.
// Conversions to/from the ark-ff form (x * 2^256 mod r, 8 x 32-bit limbs):
// from: repack bits, Montgomery-multiply by 2^266 mod r (x 2^5);
// to:   Montgomery-multiply by 2^256 mod r (x 2^-5), reduce to [0, r), repack.
#pragma once
#include "dbg_bounds.hpp"
#include "fr.hpp"

namespace lsp {

struct F29 {
    uint32_t l[9];
};

#define F29_MASK 0x1fffffffu

// r in 29-bit limbs: r[0] = 1 (r = 1 mod 2^47), r[2] = 0x42
__device__ __forceinline__ constexpr uint32_t p29(int i) {
    return i == 0 ? 0x1u
         : i == 1 ? 0x108c0000u
         : i == 2 ? 0x42u
         : i == 3 ? 0x14edfda0u
         : i == 4 ? 0x1b00159au
         : i == 5 ? 0x68f2e1bu
         : i == 6 ? 0x155982d1u
         : i == 7 ? 0xbd34594u
                  : 0x12ab65u;
}

#if defined(__HIP_DEVICE_COMPILE__) && !defined(LSP_F29_NO_ASM)
// the same product / square as ONE asm statement (tools/gen_fr29mul.py --block):
// the compiler puts a conservative s_nop after every asm statement whose result
// the next instruction reads, ~25 per product with one statement per column
// (LSP_F29_COLUMNS, gen_fr29mul.py); the single statement has none -- 7 % less
// single-wave latency (narrow Merkle levels), the same throughput
#ifdef LSP_F29_COLUMNS
#include "fr29_mul_gfx950.inc"
#else
#include "fr29_mul_gfx950_blk.inc"
#endif
#define LSP_F29_USE_ASM 1
#endif

// C = (2^261 - 1) mod r in 29-bit limbs: the constant the folded quotient
// digits below add to every product (tools/gen_fr29mul.py C29)
__device__ __forceinline__ constexpr uint32_t c29(int i) {
    return i == 0 ? 0x1ffffe49u
         : i == 1 ? 0x1077ffffu
         : i == 2 ? 0x1fff8e31u
         : i == 3 ? 0x10d0103fu
         : i == 4 ? 0xddb0965u
         : i == 5 ? 0x7071c5cu
         : i == 6 ? 0x18da2e10u
         : i == 7 ? 0x486f3a3u
         : i == 8 ? 0xec090u
                  : 0u;
}

// Montgomery product a * b * 2^-261 mod r.  FIPS, one 64-bit accumulator.
// r = 1 mod 2^29, so the quotient digit of column k can be any m'_k with
// acc + m'_k = -1 mod 2^29.  We take m'_k = ~acc mod 2^32 (a full word: no
// mask, and m'_k * r[0] = m'_k is never multiplied): acc + m'_k =
// (acc_hi + 1) 2^32 - 1, whose floor by 2^29 -- the carry -- is acc_hi * 8 + 7
// (one MAD of the high word, which also adds the next column's constant).
// Every low column of T = a b + C + M' r then ends in 29 one-bits, so the upper
// columns yield Q = (T + 1) / 2^261 - 1, and with C = (2^261 - 1) mod r (added
// limb by limb through the carries) Q == a b 2^-261 (mod r).
// Column sums stay < 2^63.2 (tools/gen_fr29mul.py --bound); M' < 2^264, so the
// output is < a b / 2^261 + 8 r + 1.
__device__ __forceinline__ F29 f29_mul_c(const F29& a, const F29& b) {
    uint32_t m[9];
    F29 o;
    uint64_t acc = c29(0);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
#pragma unroll
        for (int j = 0; j < k; ++j) {
            acc += (uint64_t)a.l[j] * b.l[k - j];
            acc += (uint64_t)m[j] * p29(k - j);
        }
        acc += (uint64_t)a.l[k] * b.l[0];
        m[k] = ~(uint32_t)acc;
        acc = (acc >> 32) * 8 + 7 + c29(k + 1);
    }
#pragma unroll
    for (int k = 9; k < 17; ++k) {
#pragma unroll
        for (int j = k - 8; j < 9; ++j) {
            acc += (uint64_t)a.l[j] * b.l[k - j];
            acc += (uint64_t)m[j] * p29(k - j);
        }
        o.l[k - 9] = (uint32_t)acc & F29_MASK;
        acc >>= 29;
    }
    o.l[8] = (uint32_t)acc;
    return o;
}

// Montgomery square: cross products a_i a_j (i < j) taken once against the
// doubled limb 2 a_i (< 2^30, products < 2^59): 45 + 72 products instead of
// 81 + 72.  Column bound: <= 5 such products + 8 m*r products + carry < 2^62.
__device__ __forceinline__ F29 f29_sqr_c(const F29& a) {
    uint32_t m[9], d[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) d[i] = a.l[i] << 1;
    F29 o;
    uint64_t acc = c29(0);
#pragma unroll
    for (int k = 0; k < 17; ++k) {
#pragma unroll
        for (int i = (k > 8 ? k - 8 : 0); 2 * i < k; ++i) acc += (uint64_t)d[i] * a.l[k - i];
        if ((k & 1) == 0) acc += (uint64_t)a.l[k / 2] * a.l[k / 2];
#pragma unroll
        for (int j = (k > 8 ? k - 8 : 0); j < (k < 9 ? k : 9); ++j) acc += (uint64_t)m[j] * p29(k - j);
        if (k < 9) {
            m[k] = ~(uint32_t)acc;
            acc = (acc >> 32) * 8 + 7 + c29(k + 1);
        } else {
            o.l[k - 9] = (uint32_t)acc & F29_MASK;
            acc >>= 29;
        }
    }
    o.l[8] = (uint32_t)acc;
    return o;
}

__device__ __forceinline__ F29 f29_mul(const F29& a, const F29& b) {
#ifdef LSP_F29_USE_ASM
    return f29_mul_asm(a, b);
#else
    return f29_mul_c(a, b);
#endif
}

__device__ __forceinline__ F29 f29_sqr(const F29& a) {
#ifdef LSP_F29_USE_ASM
    return f29_sqr_asm(a);
#else
    return f29_sqr_c(a);
#endif
}

// limb-wise sum + carry propagation (no modular reduction)
__device__ __forceinline__ F29 f29_add(const F29& a, const F29& b) {
    F29 o;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t s = a.l[i] + b.l[i] + c;
        o.l[i] = s & F29_MASK;
        c = s >> 29;
    }
    o.l[8] = a.l[8] + b.l[8] + c;
    return o;
}

// value - q*r for the small q estimated from the top limb, so that the result
// is < 2r for any input < 2^261 (q_est <= floor(v / r) <= q_est + 1)
__device__ __forceinline__ F29 f29_reduce(const F29& a) {
    // r / 2^232 = 1223525.37; q = floor(l8 / 1223526) never exceeds floor(v / r)
    // and leaves v - q r < 2r (checked exhaustively over l8 in tests/ubench)
    const uint32_t q = (uint32_t)(((uint64_t)a.l[8] * 0xdb651d12ull) >> 52);
    F29 o;
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int64_t s = (int64_t)a.l[i] - (int64_t)q * p29(i) + c;
        o.l[i] = (uint32_t)s & F29_MASK;
        c = s >> 29;  // arithmetic shift: signed carry
    }
    o.l[8] = (uint32_t)((int64_t)a.l[8] - (int64_t)q * p29(8) + c);
    return o;
}

// v - q r as f29_reduce, with q r taken from a per-workgroup LDS table
// (f29_qtab_init) instead of 64-bit multiply-and-shift chains: 3 plain 32-bit
// ops per limb instead of ~5 (two of them 64-bit), about half the VALU cycles.
// Entries hold biased limbs so every partial sum stays in [0, 2^32) and the
// carries are logical shifts: T_0 = 2^30 - Q_0, T_i = 2^30 - 2 - Q_i
// (i = 1..7), T_8 = -2 - Q_8 (mod 2^32) for Q = q r in normalised limbs; the
// running carry (s_i >> 29) is the true carry + 2, which the next entry's -2
// cancels.  Valid for values < 64 r (q <= 63) with limbs < 2.41 2^30; result
// normalised and < 2 r (the same value f29_reduce returns).
constexpr uint32_t F29_QTAB_N = 64;

// fill the table (F29_QTAB_N entries in three planes: limbs 0-3 at t[q], limbs
// 4-7 at t[F29_QTAB_N + q], limb 8 at ((uint32_t*)(t + 2 F29_QTAB_N))[q]; 2.25 KiB
// of the 3 KiB callers reserve); the caller's next __syncthreads publishes it.
// Planes, not 48-byte entries: a wave's quotients q index the limb-8 words at
// 4-byte stride, so lanes with distinct q < 32 hit distinct ds_read_b32 banks
// (the 48-byte stride repeated banks every 8 values of q; tools/lds_banks.py)
__device__ __forceinline__ void f29_qtab_init(uint4* t) {
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
        uint32_t T[9];
        T[0] = (1u << 30) - Q[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) T[i] = (1u << 30) - 2u - Q[i];
        T[8] = 0u - 2u - Q[8];
#ifdef LSP_QT_INTERLEAVED  // A/B switch (tools/variant_lib.py): round 5's 48-byte entries
        t[3 * q] = make_uint4(T[0], T[1], T[2], T[3]);
        t[3 * q + 1] = make_uint4(T[4], T[5], T[6], T[7]);
        t[3 * q + 2] = make_uint4(T[8], 0u, 0u, 0u);
#else
        t[q] = make_uint4(T[0], T[1], T[2], T[3]);
        t[F29_QTAB_N + q] = make_uint4(T[4], T[5], T[6], T[7]);
        reinterpret_cast<uint32_t*>(t + 2 * F29_QTAB_N)[q] = T[8];
#endif
    }
}

__device__ __forceinline__ F29 f29_reduce_qt(const F29& a, const uint4* __restrict__ t) {
    uint32_t q = __umulhi(a.l[8], 0xdb651d12u) >> 20;  // as f29_reduce
    // a value outside the documented bounds (top limb too large) would index past the table
    if (!LSP_BOUNDS(q < F29_QTAB_N)) q = 0;
#ifdef LSP_QT_INTERLEAVED
    const uint4 x = t[3 * q], y = t[3 * q + 1];
    const uint32_t z = reinterpret_cast<const uint32_t*>(t + 3 * q + 2)[0];
#else
    const uint4 x = t[q], y = t[F29_QTAB_N + q];
    const uint32_t z = reinterpret_cast<const uint32_t*>(t + 2 * F29_QTAB_N)[q];
#endif
    const uint32_t T[9] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, z};
    F29 o;
    uint32_t k = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t s = a.l[i] + T[i] + k;
        o.l[i] = s & F29_MASK;
        k = s >> 29;
    }
    o.l[8] = a.l[8] + T[8] + k;
    return o;
}

__device__ __forceinline__ F29 f29_zero() {
    F29 z;
#pragma unroll
    for (int i = 0; i < 9; ++i) z.l[i] = 0;
    return z;
}

// limb-wise sums without carry propagation (callers bound the limbs)
__device__ __forceinline__ F29 f29_lazy2(const F29& a, const F29& b) {
    F29 o;
#pragma unroll
    for (int i = 0; i < 9; ++i) o.l[i] = a.l[i] + b.l[i];
    return o;
}

__device__ __forceinline__ F29 f29_lazy3(const F29& a, const F29& b, const F29& c) {
    F29 o;
#pragma unroll
    for (int i = 0; i < 9; ++i) o.l[i] = a.l[i] + b.l[i] + c.l[i];
    return o;
}

// a + 16 r - b, limb-wise without carries: 16 r is held with every low limb in
// [2^29, 2^30) (borrowed from the limb above), so each difference is >= 0 for
// normalised b with value < 16 r.  Limbs < 1.5 2^30: valid as one operand of a
// product whose other operand is normalised (column sums < 2^63.5).
__device__ __forceinline__ F29 f29_sub16(const F29& a, const F29& b) {
    // 16 r (tools/gen_fr29mul.py --bound prints the derivation's check)
    constexpr uint32_t L[9] = {0x20000010u, 0x28bfffffu, 0x20000427u, 0x2edfd9ffu, 0x300159a9u,
                               0x28f2e1bcu, 0x35982d12u, 0x3d345949u, 0x12ab654u};
    F29 o;
#pragma unroll
    for (int i = 0; i < 9; ++i) o.l[i] = a.l[i] + L[i] - b.l[i];
    return o;
}

// x < 2^256 as 8 x 32-bit words -> 9 x 29-bit limbs (same integer)
__device__ __forceinline__ F29 f29_repack_in(const Fr& x) {
    F29 o;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const int bit = 29 * i, w = bit >> 5, s = bit & 31;
        uint64_t v = x.v[w];
        if (w + 1 < 8) v |= (uint64_t)x.v[w + 1] << 32;
        o.l[i] = (uint32_t)(v >> s) & (i < 8 ? F29_MASK : 0xffffffffu);
    }
    return o;
}

__device__ __forceinline__ Fr f29_repack_out(const F29& a) {
    Fr o;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const int bit = 32 * w;
        const int i = bit / 29, s = bit % 29;
        uint64_t v = (uint64_t)a.l[i] >> s;
        if (i + 1 < 9) v |= (uint64_t)a.l[i + 1] << (29 - s);
        if (i + 2 < 9) v |= (uint64_t)a.l[i + 2] << (58 - s);
        o.v[w] = (uint32_t)v;
    }
    return o;
}

__device__ __forceinline__ F29 f29_const(uint32_t l0, uint32_t l1, uint32_t l2, uint32_t l3, uint32_t l4, uint32_t l5,
                                         uint32_t l6, uint32_t l7, uint32_t l8) {
    F29 o;
    o.l[0] = l0; o.l[1] = l1; o.l[2] = l2; o.l[3] = l3; o.l[4] = l4;
    o.l[5] = l5; o.l[6] = l6; o.l[7] = l7; o.l[8] = l8;
    return o;
}

// ark-ff Montgomery (X = x 2^256 mod r, < 2^256) -> F29 (x 2^261): the integer
// X * 2^5 (< 32 r < 2^261) is already a lazily reduced F29 value, so this is a
// repack with a 5-bit offset plus one cheap reduction to < 2r -- no product.
__device__ __forceinline__ F29 f29_from_fr_lazy(const Fr& x);
__device__ __forceinline__ F29 f29_from_fr(const Fr& x) { return f29_reduce(f29_from_fr_lazy(x)); }

// X * 2^5 as F29 limbs, < 32 r, not reduced
__device__ __forceinline__ F29 f29_from_fr_lazy(const Fr& x) {
    F29 o;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const int bit = 29 * i - 5;  // limb i of X << 5 = bits [29 i - 5, 29 i + 24) of X
        uint32_t v;
        if (bit < 0) {
            v = x.v[0] << 5;
        } else {
            const int w = bit >> 5, sh = bit & 31;
            uint64_t t = x.v[w];
            if (w + 1 < 8) t |= (uint64_t)x.v[w + 1] << 32;
            v = (uint32_t)(t >> sh);
        }
        o.l[i] = v & (i < 8 ? F29_MASK : 0xffffffffu);
    }
    return o;
}

// F29 -> canonical ark-ff Montgomery words: times 2^-5 (product by 2^256 mod r), reduce to [0, r).
// Any normalised x < 2^261 is a valid operand (product < x c / 2^261 + 8r + 1 < 9r + 1), so
// no reduction before the product.
__device__ __forceinline__ Fr f29_to_fr(const F29& x) {
    const F29 c = f29_const(0x1ffffff3u, 0x8e3ffffu, 0x1ffffc9fu, 0xfea1edfu, 0xfee725u, 0xabaa896u, 0xa745b60u,
                            0x6457773u, 0xd4bdau);
    const F29 y = f29_reduce(f29_mul(x, c));  // < 2 r
    return fr_reduce_once(f29_repack_out(y));
}

// f29_to_fr with the reduction through the LDS table of q r (f29_reduce_qt:
// 32-bit ops only; identical result; the product is < 9r + 1, so q <= 8) for
// kernels that hold the table.  (Absorbed inputs keep f29_from_fr: a caller's
// word may be any value below 2^256, beyond the table's 64 r.)
__device__ __forceinline__ Fr f29_to_fr_qt(const F29& x, const uint4* __restrict__ qt) {
    const F29 c = f29_const(0x1ffffff3u, 0x8e3ffffu, 0x1ffffc9fu, 0xfea1edfu, 0xfee725u, 0xabaa896u, 0xa745b60u,
                            0x6457773u, 0xd4bdau);
    return fr_reduce_once(f29_repack_out(f29_reduce_qt(f29_mul(x, c), qt)));
}

}  // namespace lsp
