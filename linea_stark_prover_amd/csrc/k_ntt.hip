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
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "fr29.hpp"
#include "k_common.hpp"
#include "kernels.hpp"

namespace lsp {

namespace {
// PASS_INV_FWD: the inverse transform's last pass fused with the forward's first (k_ntt_rm)
enum PassMode : int { PASS_INPLACE = 0, PASS_INV_FIRST = 1, PASS_INV_FWD = 2 };

struct NttPass {
    const Fr* src;      // PASS_INV_FIRST: caller rows; PASS_INV_FWD: X after the earlier inverse passes (or caller rows)
    ColMap src_map;     // where column c of the transform sits in src (PASS_INV_FIRST, PASS_INV_FWD)
    uint32_t no_inv;    // PASS_INV_FWD: src holds the coefficients already (no inverse stages; launch_lde_coeffs)
    Fr* dst;            // the arrays being transformed (h rows each, batch of `narr` arrays, row-major w)
    const uint4* tw;    // stage-major twiddles (launch_stage_twiddles), 29-bit limbs, 3 x uint4 per element
    const uint4* tw_inv;  // PASS_INV_FWD: the inverse transform's twiddles
    uint32_t inv_gather;  // PASS_INV_FWD: the inverse has only this pass (src = caller rows, gathered bit-reversed)
    const Fr* twist;    // PASS_INV_FWD: two-level tables per (coset[, column])
    uint32_t L1, L2;    // twist table split
    uint32_t twist_per_col;  // 1: table index k*w + c, 0: table index k
    uint32_t logH, s0, k, logL, logG, w;
    uint32_t nchunk;    // column chunks of 2^LOGCW per row
    uint32_t canon;     // 1: write canonical words (the transform's last pass)
    uint32_t xcd;       // 1: workgroup ids map to tiles XCD-aware (see k_ntt_rm)
    uint32_t twl_n;     // PASS_INV_FWD: forward twiddles cached in LDS (G (2^k - 1) entries; 0: read from tw)
    uint64_t narr;      // arrays (cosets) in dst
    const Fr* ratio;    // PASS_INV_FWD, chained twist (nullptr: off): two-level table (L1, L2) of rho^row,
                        // the ratio of consecutive coset shifts when the blocks run in order arr = bitrev(j)
    uint32_t log_narr;  // with `ratio`: log2 narr
};

// element (row, col) of a pass's source through its column map; false: a
// padding column (reads as zero)
__device__ __forceinline__ bool src_at(const ColMap& m, uint64_t H, uint32_t row, uint32_t col, size_t& idx) {
    if (m.logb == COLMAP_PLAIN) {
        const uint32_t sc = m.c0 + m.cstep * col;
        if (sc >= m.valid) return false;
        idx = (size_t)row * m.stride + sc;
        return true;
    }
    const uint32_t b = brev_bits(col & ((1u << m.logb) - 1), m.logb), c = col >> m.logb;
    idx = ((size_t)b * H + row) * m.bw + c;
    return true;
}

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

// A tile value to ark words.  Between passes the arrays keep the values as the
// stages leave them (normalised, < 8.3 r < 2^256: the invariant inside a pass,
// which the next pass's loads accept); the transform's last stage is trivial
// and reduces its outputs below 2r, so the last pass (canon) needs only one
// conditional subtraction.  No product-sized reduction on any store.
__device__ __forceinline__ Fr f29_store(const F29& v, bool canon) {
    const Fr o = f29_repack_out(v);
    return canon ? fr_reduce_once(o) : o;
}

// carry propagation only (no modular reduction): limbs < 2^32 - 2^3 in,
// limbs 0..7 < 2^29 out, same integer
__device__ __forceinline__ F29 f29_norm(const F29& a) {
    F29 o;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t s = a.l[i] + c;
        o.l[i] = s & F29_MASK;
        c = s >> 29;
    }
    o.l[8] = a.l[8] + c;
    return o;
}

// a + 32 r - b limb-wise (as f29_sub16): b normalised with value < 32 r;
// limbs < 1.5 2^30, a valid product operand up to ~60 r
// (tools/gen_fr29mul.py --bound checks the column sums)
__device__ __forceinline__ F29 f29_sub32(const F29& a, const F29& b) {
    constexpr uint32_t L[9] = {0x20000020u, 0x317fffffu, 0x2000084fu, 0x3dbfb3ffu, 0x2002b353u,
                               0x31e5c37au, 0x2b305a25u, 0x3a68b294u, 0x2556caau};
    F29 o;
#pragma unroll
    for (int i = 0; i < 9; ++i) o.l[i] = a.l[i] + L[i] - b.l[i];
    return o;
}

// The tile in LDS as three planes (limbs 0-3, limbs 4-7, limb 8), so an
// element is one ds_read_b128 + ds_read_b128 + ds_read_b32 at any index
// (a 36-byte array element is only 4-byte aligned: 5 narrow reads)
struct TileLds {
    uint4* a;
    uint4* b;
    uint32_t* c;
    __device__ __forceinline__ F29 get(uint32_t e) const {
        const uint4 x = a[e], y = b[e];
        F29 o;
        o.l[0] = x.x; o.l[1] = x.y; o.l[2] = x.z; o.l[3] = x.w;
        o.l[4] = y.x; o.l[5] = y.y; o.l[6] = y.z; o.l[7] = y.w;
        o.l[8] = c[e];
        return o;
    }
    __device__ __forceinline__ void put(uint32_t e, const F29& v) const {
        a[e] = make_uint4(v.l[0], v.l[1], v.l[2], v.l[3]);
        b[e] = make_uint4(v.l[4], v.l[5], v.l[6], v.l[7]);
        c[e] = v.l[8];
    }
};

// The LDS slot of tile element e: an XOR swizzle of its low bits by higher
// bits, e ^ ((e >> 1) & 8) ^ ((e >> 2) & 31) (bits 2..6 -> 0..4, bit 4 -> 3).
// Unswizzled, the radix-4 groups at distances 1 and 4 (and 2 and 8 with two
// columns per row) put a wave's lanes on a quarter of the banks: 14 and 8.7
// extra LDS cycles per instruction, 3.6 per LDS instruction over a pass, as
// the PMC measured (SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS 3.9 / 3.1 / 2.2,
// profiles/r05l_valu_pmc.txt).  This map makes every ds_read_b128 16-lane
// group, ds_read/write_b32 32-lane half and ds_write_b128 8-lane group of
// every radix-4 distance at 1 and 2 columns per row hit distinct banks (one
// 2-way group left, the radix-2 stage at distance 1 with 2 columns), and at
// 4 and 8 columns too (tools/lds_banks.py --swizzle ntt, found by the search
// there; of the maps that do this, the cheapest found: two shift-mask terms,
// half the VALU of the five-bit map tried first, which the fused pass paid
// for: +5 % on a VALU-bound kernel).  It is XOR-linear and moves bits only downwards, so it permutes
// [0, 2^j) for every j: the tile's size is unchanged, and a quad's members
// e0 | m de (e0 zero at de's bits) sit at tswz(e0) ^ tswz(m de), one wave-
// uniform XOR each.
//
// Measured (round 6, profiles/r06_lds_swizzle.txt): the swizzle takes the
// passes' SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS from 3.9 / 2.2 / 3.1 to 0.2 / 0.4
// / 0.2 and their LDS wait share from 6.6 / 2.8 / 3.6 to 3.4 / 1.4 / 2.1 per
// LDS instruction -- and the LDE's time not at all (2^19 x 8: 3.183 against
// 3.179 ms, medians of 8 alternating runs), while whole proofs ran 0.22-0.27
// ms slower with it (paired, both orders): the passes are VALU-bound, the
// conflicts were hidden behind the other waves' VALU work, and the map's
// instructions are not.  So the tile ships unswizzled; LSP_NTT_SWZ builds it
// (tools/variant_lib.py).
__device__ __forceinline__ uint32_t tswz(uint32_t e) {
#ifdef LSP_NTT_SWZ
    return e ^ ((e >> 1) & 8u) ^ ((e >> 2) & 31u);
#else
    return e;
#endif
}

// The fused pass's twiddle cache in LDS: 48-byte slots (limbs 0-3, 4-7, 8 +
// padding), read by f29_load48.  LSP_NTT_TWL_PLANES stores it in three planes
// as TileLds instead (36 bytes an entry, the limb-8 words at 4-byte stride, so
// distinct entries never share a ds_read_b32 bank within 32 of them): measured
// 2 % slower over the whole LDE (2^19 x 8: 3.207 against 3.131 ms,
// profiles/r06_lds_swizzle.txt), so the slots stay.
struct TwlLds {
    uint4* a;
    uint4* b;
    uint32_t* c;
#ifndef LSP_NTT_TWL_PLANES  // 48-byte slots, all in `a` (the planes are the A/B variant)
    __device__ __forceinline__ F29 get(uint32_t i) const { return f29_load48(a + 3 * i); }
    __device__ __forceinline__ void put(uint32_t i, const uint4* src) const {
        a[3 * i] = src[0];
        a[3 * i + 1] = src[1];
        a[3 * i + 2] = src[2];
    }
    static constexpr size_t BYTES = 3 * sizeof(uint4);
#else
    __device__ __forceinline__ F29 get(uint32_t i) const {
        const uint4 x = a[i], y = b[i];
        F29 o;
        o.l[0] = x.x; o.l[1] = x.y; o.l[2] = x.z; o.l[3] = x.w;
        o.l[4] = y.x; o.l[5] = y.y; o.l[6] = y.z; o.l[7] = y.w;
        o.l[8] = c[i];
        return o;
    }
    __device__ __forceinline__ void put(uint32_t i, const uint4* src) const {
        a[i] = src[0];
        b[i] = src[1];
        c[i] = src[2].x;
    }
    static constexpr size_t BYTES = 2 * sizeof(uint4) + sizeof(uint32_t);
#endif
};

// Two radix-2 stages in registers (radix-4 groups): per group 4 elements are
// read from and written to the LDS once instead of twice, one barrier per two
// stages, 3 twiddles per 4 butterflies, and the sums between the two stages
// only carry-normalised.  Invariant between groups: normalised and < 8.3 r.
//
// DIF stages s (distance D) and s + 1 (D/2) on v0..v3 = positions t0, t0 + D/2,
// t0 + D, t0 + 3D/2: wA = w(s, t0), wA2 = w(s, t0 + D/2), wB = w(s + 1, t0)
// (= w(s + 1, t0 + D)); TRIV: stage s + 1 is the transform's last (w = 1).
// u0 stays carry-free (limbs < 2^30): as the minuend of f29_sub32 it makes
// limbs < 2^31 and column sums < 2^63.74 in the product by wB
// (tools/gen_fr29mul.py --bound), and f29_reduce takes it as it is (its
// quotient estimate from the top limb still leaves < 2r).
// the reductions of a group: f29_reduce, or with a per-workgroup LDS table of
// q r (f29_reduce_qt: 3 plain 32-bit ops per limb instead of 64-bit
// multiply-adds and shifts) when qt is given.  Every reduced sum below is
// < 64 r with limbs < 2^31 (the table's biased limb sums stay in [0, 2^32)
// up to limbs of 3 2^30; its top-limb quotient estimate leaves < 2r as f29_reduce's).
__device__ __forceinline__ F29 red(const F29& v, const uint4* __restrict__ qt) {
    return qt ? f29_reduce_qt(v, qt) : f29_reduce(v);
}

template <bool TRIV>
__device__ __forceinline__ void dif4(F29& v0, F29& v1, F29& v2, F29& v3, const F29& wA, const F29& wA2,
                                     const F29& wB, const uint4* __restrict__ qt) {
    const F29 u0 = f29_lazy2(v0, v2);                  // < 16.6 r, limbs < 2^30
    const F29 u1 = f29_norm(f29_lazy2(v1, v3));
    const F29 u3 = f29_mul(f29_sub16(v1, v3), wA2);
    if constexpr (TRIV) {
        // the transform's last two stages: the group starts at an even row, so
        // wA = w_4^0 = 1 as well and u2 needs no product.  u2 = sub16(v0, v2):
        // limbs < 1.5 2^30, < 24.3 r; sub16(u2, u3) is dit4's sub16 of a sub16
        // (limbs < 2.42 2^30, < 40.3 r), which both reductions take
        const F29 u2 = f29_sub16(v0, v2);
        v0 = red(f29_lazy2(u0, u1), qt);
        v2 = red(f29_lazy2(u2, u3), qt);
        v1 = red(f29_sub32(u0, u1), qt);
        v3 = red(f29_sub16(u2, u3), qt);
    } else {
        const F29 u2 = f29_mul(f29_sub16(v0, v2), wA);  // < 8.06 r
        v0 = red(f29_lazy2(u0, u1), qt);                // < 2 r
        v2 = red(f29_lazy2(u2, u3), qt);
        v1 = f29_mul(f29_sub32(u0, u1), wB);            // < 48.6 r in -> < 8.11 r
        v3 = f29_mul(f29_sub16(u2, u3), wB);
    }
}

// DIT stages s (distance d) and s + 1 (2d) on v0..v3 = positions t0, t0 + d,
// t0 + 2d, t0 + 3d: wA = w(s, t0) (= w(s, t0 + 2d)), wB = w(s + 1, t0),
// wB2 = w(s + 1, t0 + d); TRIV: stage s is the transform's first (w = 1).
template <bool TRIV>
__device__ __forceinline__ void dit4(F29& v0, F29& v1, F29& v2, F29& v3, const F29& wA, const F29& wB,
                                     const F29& wB2, const uint4* __restrict__ qt) {
    if constexpr (TRIV) {
        // the transform's first two stages: the group starts at a row = 0 mod 4,
        // so wB = w_4^0 = 1 as well.  u2 = v2 + v3 is normalised (< 16.6 r) to be
        // the subtrahend of f29_sub32 (u0 + 32 r - u2: limbs < 2^31, < 48.6 r)
        const F29 u0 = f29_lazy2(v0, v1);
        const F29 u1 = f29_sub16(v0, v1);
        const F29 u2 = f29_norm(f29_lazy2(v2, v3));
        const F29 q3 = f29_mul(f29_sub16(v2, v3), wB2);
        v0 = red(f29_lazy2(u0, u2), qt);
        v2 = red(f29_sub32(u0, u2), qt);
        v1 = red(f29_lazy2(u1, q3), qt);
        v3 = red(f29_sub16(u1, q3), qt);
    } else {
        const F29 p1 = f29_mul(v1, wA);                 // < 8.3 r
        const F29 p3 = f29_mul(v3, wA);
        const F29 u0 = f29_lazy2(v0, p1);               // limbs < 2^30, < 16.6 r
        const F29 u1 = f29_sub16(v0, p1);               // limbs < 1.5 2^30, < 24.6 r
        const F29 u2 = f29_lazy2(v2, p3);
        const F29 u3 = f29_sub16(v2, p3);
        const F29 q2 = f29_mul(u2, wB);                 // < 8.07 r
        const F29 q3 = f29_mul(u3, wB2);
        v0 = red(f29_lazy2(u0, q2), qt);                // < 2 r
        v2 = red(f29_sub16(u0, q2), qt);
        v1 = red(f29_lazy2(u1, q3), qt);
        v3 = red(f29_sub16(u1, q3), qt);                // limbs < 2.42 2^30
    }
}

// One tile: 2^k positions x 2^logG groups x 2^LOGCW columns (power-of-two
// chunk, so every index below is shifts and masks; rows are 32-bit within
// an array, H <= 2^31).  The first forward pass runs one workgroup per tile of
// the coefficients for ALL cosets: the tile is kept in registers (<= 4
// elements per thread) and twisted, transformed and stored once per coset, so
// the coefficients are not re-read for every coset.  That pass is fused with
// the inverse transform's last pass, which covers the same rows (stride
// 2^(logH - k)): the coefficients never go to HBM.
constexpr uint32_t NTT_THREADS = 256;
constexpr uint32_t NTT_MAX_EL = 1024;  // 2^k x G x CW
__device__ __forceinline__ uint32_t k_pos(uint32_t k) { return 1u << k; }  // positions of a tile

template <int LOGCW>
struct TileGeom {
    uint32_t k, logG, logL, gid0;
    __device__ __forceinline__ uint32_t row_of(uint32_t t, uint32_t g) const {
        const uint32_t gid = gid0 + g;
        return ((gid >> logL) << (logL + k)) + (t << logL) + (gid & ((1u << logL) - 1));
    }
    // element e of a thread-strided loop -> (position, group, column)
    __device__ __forceinline__ void split(uint32_t e, uint32_t& t, uint32_t& g, uint32_t& c) const {
        c = e & ((1u << LOGCW) - 1);
        const uint32_t tg = e >> LOGCW;
        if (logL < logG) {  // rows of adjacent positions are adjacent: position fastest
            t = tg & ((1u << k) - 1);
            g = tg >> k;
        } else {
            t = tg >> logG;
            g = tg & ((1u << logG) - 1);
        }
    }
    __device__ __forceinline__ uint32_t idx(uint32_t t, uint32_t g, uint32_t c) const {
        return (((t << logG) + g) << LOGCW) + c;
    }
};

// The fused pass's forward twiddles, cached in LDS once per workgroup: its
// tile rows are t 2^logL + gid (s0 = 0, logL + k = logH), so DIF stage s < k
// reads w^(gid + (t mod 2^(k-1-s)) 2^logL) -- 2^(k-1-s) distinct values per row
// group, G (2^k - 1) for the tile.  Read from the global table they were
// fetched again for every coset (the tile's twiddles outgrow the L2 across the
// workgroups of an XCD); from LDS, once.  Entry of (group g, stage s, u):
// g (2^k - 1) + (2^k - 2^(k-s)) + u.
template <int LOGCW>
__device__ __forceinline__ uint32_t twl_index(const TileGeom<LOGCW>& gm, uint32_t row, uint32_t s) {
    const uint32_t k = gm.k;
    const uint32_t u = (row >> gm.logL) & ((1u << (k - 1 - s)) - 1);
    const uint32_t g = (row & ((1u << gm.logL) - 1)) - gm.gid0;
    return g * ((1u << k) - 1) + ((1u << k) - (1u << (k - s))) + u;
}

// stages s0 .. s0 + k - 1 of the tile in LDS: radix-4 groups of two stages,
// then a radix-2 stage if k is odd; ends with a barrier
template <bool DIF, int LOGCW>
__device__ __forceinline__ void tile_stages(const TileLds& T, const TileGeom<LOGCW>& gm, const uint4* __restrict__ tw,
                                            uint32_t s0, uint32_t logH, uint32_t n_el,
                                            TwlLds twl = TwlLds{nullptr, nullptr, nullptr},
                                            const uint4* qt = nullptr, uint32_t twl_n = 0) {
    constexpr uint32_t CW = 1u << LOGCW;
    const uint32_t k = gm.k, G = 1u << gm.logG;
    const uint32_t cshift = gm.logG + LOGCW;  // element index = (t << cshift) + (g << LOGCW) + c
    const uint64_t H = 1ull << logH;
    auto tw_at = [&](uint32_t row, uint32_t s) -> F29 {
        // stage s uses the powers of w_(2^m), m = logH - s (DIF) or s + 1 (DIT):
        // DIF w^((row mod H/2^(s+1)) 2^s), DIT w^((row mod 2^s) 2^(logH-1-s)); the
        // table is stage-major (entry 2^(m-1) - 1 + i = w_(2^m)^i), so
        // consecutive rows read consecutive slots
        if (DIF && twl_n) {  // the fused pass's LDS copy
            const uint32_t ti = twl_index(gm, row, s);
            return twl.get(LSP_BOUNDS(ti < twl_n) ? ti : 0u);
        }
        const uint32_t half = DIF ? (uint32_t)(H >> (s + 1)) : (1u << s);
        if (!LSP_BOUNDS(s < logH && row < H)) return f29_zero();
        return f29_load48(tw + 3 * (size_t)(half - 1 + (row & (half - 1))));
    };
    uint32_t j = 0;
    for (; j + 1 < k; j += 2) {
        const uint32_t s = s0 + j;
        // the quad's members are t0 + m 2^b: DIF distances 2^(b+1), 2^b; DIT 2^b, 2^(b+1)
        const uint32_t b = DIF ? (k - 2 - j) : j;
        const uint32_t bmask = (1u << b) - 1;
        // the group at the transform's trivial end (the DIT's first two stages,
        // the DIF's last two) runs its own loop: one product instead of four
        // (dif4 / dit4 with TRIV), and its own register allocation
        auto groups = [&](auto triv_tag) {
            constexpr bool TRIV = decltype(triv_tag)::value;
            for (uint32_t qd = threadIdx.x; qd < (n_el >> 2); qd += NTT_THREADS) {
                const uint32_t c = qd & (CW - 1);
                const uint32_t pg = qd >> LOGCW;
                const uint32_t g = pg & (G - 1), pp = pg >> gm.logG;
                const uint32_t t0 = ((pp & ~bmask) << 2) | (pp & bmask);
                const uint32_t e0 = (t0 << cshift) + (g << LOGCW) + c, de = (1u << b) << cshift;
                if (!LSP_BOUNDS(e0 + 3 * de < n_el && t0 + 3 * (1u << b) < k_pos(k))) continue;
                // e0 is zero at de's two bits: member m sits at tswz(e0) ^ tswz(m de)
                const uint32_t x0 = tswz(e0), d1 = tswz(de), d2 = tswz(2 * de);
                const uint32_t x1 = x0 ^ d1, x2 = x0 ^ d2, x3 = x1 ^ d2;
                F29 v0 = T.get(x0), v1 = T.get(x1), v2 = T.get(x2), v3 = T.get(x3);
                const uint32_t r0 = gm.row_of(t0, g), dr = (1u << b) << gm.logL;
                if constexpr (DIF) {
                    if constexpr (TRIV)
                        dif4<true>(v0, v1, v2, v3, v0, tw_at(r0 + dr, s), v0, qt);
                    else
                        dif4<false>(v0, v1, v2, v3, tw_at(r0, s), tw_at(r0 + dr, s), tw_at(r0, s + 1), qt);
                } else {
                    if constexpr (TRIV)
                        dit4<true>(v0, v1, v2, v3, v0, v0, tw_at(r0 + dr, s + 1), qt);
                    else
                        dit4<false>(v0, v1, v2, v3, tw_at(r0, s), tw_at(r0, s + 1), tw_at(r0 + dr, s + 1), qt);
                }
                T.put(x0, v0);
                T.put(x1, v1);
                T.put(x2, v2);
                T.put(x3, v3);
            }
        };
        if (DIF ? (s + 1 == logH - 1) : (s == 0))
            groups(std::true_type{});
        else
            groups(std::false_type{});
        __syncthreads();
    }
    if (j < k) {  // the last stage alone (odd k)
        const uint32_t s = s0 + j;
        const uint32_t logd = DIF ? 0u : j;
        const bool trivial = DIF ? (s == logH - 1) : (s == 0);
        const uint32_t dmask = (1u << logd) - 1;
        for (uint32_t bf = threadIdx.x; bf < (n_el >> 1); bf += NTT_THREADS) {
            const uint32_t c = bf & (CW - 1);
            const uint32_t pg = bf >> LOGCW;
            const uint32_t g = pg & (G - 1), pp = pg >> gm.logG;
            const uint32_t t0 = ((pp >> logd) << (logd + 1)) | (pp & dmask);
            const uint32_t e0 = (t0 << cshift) + (g << LOGCW) + c, e1 = e0 + ((1u << logd) << cshift);
            if (!LSP_BOUNDS(e1 < n_el)) continue;
            const uint32_t a0 = tswz(e0), a1 = a0 ^ tswz((1u << logd) << cshift);  // e0 zero at that bit
            const F29 a = T.get(a0), b = T.get(a1);
            if (trivial) {
                T.put(a0, red(f29_lazy2(a, b), qt));
                T.put(a1, red(f29_sub16(a, b), qt));
                continue;
            }
            const F29 wv = tw_at(gm.row_of(t0, g), s);
            if (DIF) {
                T.put(a0, red(f29_lazy2(a, b), qt));
                T.put(a1, f29_mul(f29_sub16(a, b), wv));
            } else {
                const F29 bw = f29_mul(b, wv);
                T.put(a0, red(f29_lazy2(a, bw), qt));
                T.put(a1, red(f29_sub16(a, bw), qt));
            }
        }
        __syncthreads();
    }
}

template <bool DIF, int MODE, int LOGCW>
__global__ __launch_bounds__(NTT_THREADS) void k_ntt_rm(NttPass p) {
    extern __shared__ uint4 lds_raw[];
    constexpr uint32_t CW = 1u << LOGCW;
    constexpr bool FWD_FIRST = MODE == PASS_INV_FWD;
    const uint32_t K = 1u << p.k, logG = p.logG;
    const uint64_t H = 1ull << p.logH;
    const uint32_t tiles_per_arr = (uint32_t)(H >> (p.k + logG)) * p.nchunk;
    // Workgroups are dispatched round-robin over the 8 XCDs (each with its own
    // L2).  With narrow column chunks a row's 256 bytes are read by nchunk
    // workgroups: give all chunks of one tile to one XCD, back to back, so the
    // row's lines are fetched from HBM once and served from that XCD's L2.
    uint32_t wg = blockIdx.x;
    if (p.xcd) {
        const uint32_t x = wg & 7, i = wg >> 3;
        const uint32_t tl = i / p.nchunk;
        wg = ((tl << 3) + x) * p.nchunk + (i - tl * p.nchunk);
    }
    const uint32_t arr0 = FWD_FIRST ? 0u : wg / tiles_per_arr;
    const uint32_t arr_end = FWD_FIRST ? (uint32_t)p.narr : arr0 + 1;
    const uint32_t rem = wg - arr0 * tiles_per_arr;
    const uint32_t tile = rem / p.nchunk;
    const uint32_t c0 = (rem - tile * p.nchunk) << LOGCW;
    const uint32_t cw = min(CW, p.w - c0);
    const uint32_t n_el = (K << logG) << LOGCW;
    const TileGeom<LOGCW> gm{p.k, logG, p.logL, tile << logG};
    const TileLds T{lds_raw, lds_raw + n_el, reinterpret_cast<uint32_t*>(lds_raw + 2 * n_el)};
    // the reduction table after the tile (3 KiB; not in the fused pass, whose
    // LDS already limits it to 2 workgroups per CU); published by the barrier
    // after the tile's load below
    const uint4* qt = nullptr;
#ifndef LSP_NTT_NO_QT  // A/B switch (tools/variant_lib.py): f29_reduce everywhere
    if constexpr (!FWD_FIRST) {
        uint4* q = reinterpret_cast<uint4*>(T.c + n_el);
        f29_qtab_init(q);
        qt = q;
    }
#endif
    constexpr uint32_t NREG = FWD_FIRST ? NTT_MAX_EL / NTT_THREADS : 1;
    F29 xr[NREG];
    uint32_t xs[NREG];  // the fused pass: the LDS slots of this thread's elements, for every coset
    // the forward twiddles of this tile in LDS (after the tile and the per-row
    // twist factors; published by the barrier after the coefficient load below)
    // (by value: a pointer to it would put the struct in scratch memory)
    TwlLds twl{nullptr, nullptr, nullptr};
    if (FWD_FIRST && p.twl_n) {
        const bool rt = !p.twist_per_col || p.ratio;  // the row factors sit between the tile and these
        const size_t off = (size_t)n_el * sizeof(F29) + (rt ? (size_t)(K << logG) * sizeof(F29) : 0);
        uint4* base = reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds_raw) + ((off + 15) & ~(size_t)15));
        twl = TwlLds{base, base + p.twl_n, reinterpret_cast<uint32_t*>(base + 2 * p.twl_n)};
        const uint32_t per = K - 1;  // entries per row group
        for (uint32_t e = threadIdx.x; e < p.twl_n; e += NTT_THREADS) {
            const uint32_t g = e / per, r = e - g * per;
            const uint32_t m = K - r;                       // 1 .. 2^k: stage s has m in (2^(k-1-s), 2^(k-s)]
            const uint32_t s = p.k - (32 - __builtin_clz(m - 1 + (m == 1)));  // k - ceil(log2 m)
            const uint32_t sk = m == 1 ? p.k - 1 : s;
            const uint32_t u = r - (K - (K >> sk));
            const uint32_t half = (uint32_t)(H >> (sk + 1));
            const size_t gi = (size_t)(half - 1) + gm.gid0 + g + ((size_t)u << p.logL);
            if (!LSP_BOUNDS(gi + 1 < H && sk < p.k)) continue;
            twl.put(e, p.tw + 3 * gi);
        }
    }
    if (FWD_FIRST) {
        // ---- the inverse transform's last stages over these rows (logH - k ..
        // logH - 1; from the caller's rows, gathered bit-reversed, when the
        // inverse has only this pass), then the coefficients (x h) stay in registers
        for (uint32_t e = threadIdx.x; e < n_el; e += NTT_THREADS) {
            uint32_t t, g, c;
            gm.split(e, t, g, c);
            if (c >= cw) {  // padding columns of the last chunk: zeros (the butterflies reduce them too)
                T.put(tswz(gm.idx(t, g, c)), f29_zero());
                continue;
            }
            const uint32_t row = gm.row_of(t, g);
            const uint32_t srow = p.inv_gather ? brev_bits(row, p.logH) : row;
            size_t si;
            if (!LSP_BOUNDS(row < H && gm.idx(t, g, c) < n_el && c0 + c < p.w)) continue;
            T.put(tswz(gm.idx(t, g, c)),
                  src_at(p.src_map, H, srow, c0 + c, si) ? f29_repack_in(p.src[si]) : f29_zero());
        }
        __syncthreads();
        if (!p.no_inv) tile_stages<false, LOGCW>(T, gm, p.tw_inv, p.logH - p.k, p.logH, n_el);
#pragma unroll
        for (uint32_t j = 0; j < NREG; ++j) {
            const uint32_t e = threadIdx.x + j * NTT_THREADS;
            uint32_t t, g, c;
            gm.split(e, t, g, c);
            xs[j] = tswz(gm.idx(t, g, c));
            if (e < n_el && c < cw) xr[j] = T.get(xs[j]);  // normalised, < 8.3 r
        }
    }
    F29* fac = reinterpret_cast<F29*>(T.c + n_el);  // K * G extra entries (launcher sizes the LDS for it)
    const bool row_twist = FWD_FIRST && !p.twist_per_col;
    // Chained twist: coset blocks run in the order arr = bitrev(j), whose shifts
    // are s rho^j, so block j's twisted coefficients are block j-1's times
    // rho^row -- one product per element and block (the registers carry the
    // running value) instead of the twist plus its factor from the two-level
    // table.  rho^row is a row factor shared by every column, in `fac` from j = 1.
    const bool chain = FWD_FIRST && p.ratio != nullptr;
    for (uint32_t j = arr0; j < arr_end; ++j) {
        const uint32_t arr = chain ? (uint32_t)brev_bits(j, p.log_narr) : j;
        if (!LSP_BOUNDS(arr < p.narr)) return;
        Fr* base = p.dst + (size_t)arr * H * p.w;
        if (FWD_FIRST) __syncthreads();  // the previous reads of the tile (and of fac) are done
        // ---- row factors (29-bit form): s^row / h once per row when every column
        // shares the shift; with the chain, rho^row (computed once, at j = 1)
        if (chain ? (j == 1 || (j == 0 && row_twist)) : row_twist) {
            const Fr* tab = chain && j == 1 ? p.ratio : p.twist + (size_t)arr * ((1ull << p.L1) + (1ull << p.L2));
            for (uint32_t rg = threadIdx.x; rg < (K << logG); rg += NTT_THREADS) {
                uint32_t t, g, c;
                gm.split(rg << LOGCW, t, g, c);
                if (!LSP_BOUNDS(gm.row_of(t, g) < H && (gm.row_of(t, g) >> p.L1) < (1u << p.L2))) continue;
                fac[(t << logG) + g] = pow2l29(tab, p.L1, gm.row_of(t, g));
            }
            __syncthreads();
        }
        // ---- load (twisting the registers, or from the array)
        if (FWD_FIRST) {
#pragma unroll
            for (uint32_t jr = 0; jr < NREG; ++jr) {
                const uint32_t e = threadIdx.x + jr * NTT_THREADS;
                uint32_t t, g, c;
                gm.split(e, t, g, c);
                if (e >= n_el) continue;
                if (c >= cw) {  // padding column: zero in the tile (never stored)
                    T.put(xs[jr], f29_zero());
                    continue;
                }
                F29 f;
                if (!LSP_BOUNDS(((t << logG) + g) < (K << logG) && gm.idx(t, g, c) < n_el)) continue;
                if (row_twist || (chain && j > 0)) {
                    f = fac[(t << logG) + g];
                } else {
                    const Fr* tab = p.twist + ((size_t)arr * p.w + c0 + c) * ((1ull << p.L1) + (1ull << p.L2));
                    f = pow2l29(tab, p.L1, gm.row_of(t, g));
                }
                if (chain) {
                    xr[jr] = f29_mul(xr[jr], f);  // < 8.2 r for inputs < 8.3 r and f < r, at every step
                    T.put(xs[jr], xr[jr]);
                } else {
                    T.put(xs[jr], f29_mul(xr[jr], f));  // < 8.3 r
                }
            }
        } else {
            for (uint32_t e = threadIdx.x; e < n_el; e += NTT_THREADS) {
                uint32_t t, g, c;
                gm.split(e, t, g, c);
                if (c >= cw) {  // padding columns of the last chunk: zeros (the butterflies reduce them too)
                    T.put(tswz(gm.idx(t, g, c)), f29_zero());
                    continue;
                }
                const uint32_t row = gm.row_of(t, g);
                if (!LSP_BOUNDS(row < H && gm.idx(t, g, c) < n_el && c0 + c < p.w)) continue;
                F29 v;
                size_t si;
                if (MODE == PASS_INV_FIRST)
                    v = src_at(p.src_map, H, brev_bits(row, p.logH), c0 + c, si) ? f29_repack_in(p.src[si]) : f29_zero();
                else
                    v = f29_repack_in(base[(size_t)row * p.w + c0 + c]);
                T.put(tswz(gm.idx(t, g, c)), v);
            }
        }
        __syncthreads();
        tile_stages<DIF, LOGCW>(T, gm, p.tw, p.s0, p.logH, n_el, twl, qt, FWD_FIRST ? p.twl_n : 0u);
        // ---- store
        const bool canon = p.canon != 0;
        if constexpr (FWD_FIRST) {  // this thread's elements, at the slots computed once (xs)
#pragma unroll
            for (uint32_t jr = 0; jr < NREG; ++jr) {
                const uint32_t e = threadIdx.x + jr * NTT_THREADS;
                uint32_t t, g, c;
                gm.split(e, t, g, c);
                if (e >= n_el || c >= cw) continue;
                if (!LSP_BOUNDS(gm.row_of(t, g) < H && gm.idx(t, g, c) < n_el && c0 + c < p.w)) continue;
                base[(size_t)gm.row_of(t, g) * p.w + c0 + c] = f29_store(T.get(xs[jr]), canon);
            }
        } else {
            for (uint32_t e = threadIdx.x; e < n_el; e += NTT_THREADS) {
                uint32_t t, g, c;
                gm.split(e, t, g, c);
                if (c >= cw) continue;
                if (!LSP_BOUNDS(gm.row_of(t, g) < H && gm.idx(t, g, c) < n_el && c0 + c < p.w)) continue;
                base[(size_t)gm.row_of(t, g) * p.w + c0 + c] = f29_store(T.get(tswz(gm.idx(t, g, c))), canon);
            }
        }
    }
}

// A sub-coset's folded coefficients (launch_fold_subcoset): out[i][c] =
// sum_t coef[i + t S][c] fac[c f + t].  Inputs as the inverse leaves them
// (< 8.3 r), factors canonical in the 29-bit form; each product < 8.06 r,
// the running sum reduced below 2 r after every addition, stored < 2 r.
__global__ __launch_bounds__(256) void k_fold_subcoset(const Fr* __restrict__ coef, ColMap map, uint64_t H, uint64_t S,
                                                       uint32_t w, uint32_t f, const Fr* __restrict__ fac,
                                                       Fr* __restrict__ out) {
    const size_t e = gtid();
    if (e >= S * w) return;
    const size_t i = e / w;
    const uint32_t c = (uint32_t)(e - i * w);
    F29 acc = f29_zero();
    for (uint32_t t = 0; t < f; ++t) {
        size_t si;
        if (!src_at(map, H, (uint32_t)(i + t * S), c, si)) continue;  // a padding column
        acc = f29_reduce(f29_lazy2(acc, f29_mul(f29_repack_in(coef[si]), f29_repack_in(fac[(size_t)c * f + t]))));
    }
    out[e] = f29_store(acc, false);
}

// out[i][c] = X[i][c] f^i canonical, f^i from a two-level table of 29-bit-form
// factors (pow2l29): the coefficients of an inverse transform (h * c_i, as
// launch_intt leaves them) times (1/h) shift^-i (coset_idft_batch)
__global__ __launch_bounds__(256) void k_scale_coeffs(const Fr* __restrict__ X, size_t h, uint32_t w,
                                                      const Fr* __restrict__ tab, uint32_t L1, Fr* __restrict__ out) {
    const size_t e = gtid();
    if (e >= h * w) return;
    const size_t i = e / w;
    out[e] = f29_store(f29_reduce(f29_mul(f29_repack_in(X[e]), pow2l29(tab, L1, i))), true);
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

__global__ __launch_bounds__(256) void k_stage_twiddles(const Fr* __restrict__ pw, uint32_t logH,
                                                         uint4* __restrict__ out) {
    const size_t j = gtid();
    if (j + 1 >= (1ull << logH)) return;
    const uint32_t m = 64 - __clzll((unsigned long long)(j + 1));  // 2^(m-1) <= j + 1 < 2^m
    const size_t i = j + 1 - (1ull << (m - 1));
    const F29 v = f29_repack_in(f29_store(f29_from_fr(pw[i << (logH - m)]), true));
    out[3 * j] = make_uint4(v.l[0], v.l[1], v.l[2], v.l[3]);
    out[3 * j + 1] = make_uint4(v.l[4], v.l[5], v.l[6], v.l[7]);
    out[3 * j + 2] = make_uint4(v.l[8], 0u, 0u, 0u);
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

// the passes of an LDE (WHAT = LDE_FULL), of its inverse half only
// (LDE_INV: X <- h * coefficients) or of its forward half only (LDE_FWD: from
// h * coefficients at `in` through `map`)
enum LdeWhat { LDE_FULL = 0, LDE_INV = 1, LDE_FWD = 2 };

static hipError_t run_lde(LdeWhat what, const Fr* in, ColMap map, Fr* X, Fr* out, size_t w, uint32_t logh,
                          uint32_t ncosets, const uint4* tw_inv, const uint4* tw_fwd, const Fr* twist, uint32_t L1,
                          uint32_t L2, int twist_per_col, const Fr* ratio, hipStream_t st) {
    if (w == 0) return hipSuccess;
    uint32_t log_narr = 0;
    while ((1u << log_narr) < ncosets) ++log_narr;
    if (ratio && (ncosets < 2 || (1u << log_narr) != ncosets)) return hipErrorInvalidValue;
    // Tile = 2^k positions x G groups x CW columns = 1024 elements (36 KiB of
    // LDS) where the array allows it, so every radix-4 group gives each of the
    // 256 threads one quad.  Up to k = 10 stages per pass with one column per
    // tile (2^19 points in 2 passes instead of 3: fewer HBM round trips); a
    // pass with fewer stages takes the widest column chunk that still fits
    // (k = 9: CW = 2, ..., k <= 7: CW = 8), and the narrow row accesses are
    // merged in L2 by the XCD-aware tile order.  LSP_NTT_LOGCW (minimum column
    // chunk) / LSP_NTT_KMAX override (LOGCW=3 KMAX=7: the r01 shape).
    // minimum log2 column chunk (bounds k).  Narrow chunks rely on the XCD's L2
    // holding a tile's rows until all its chunks have read them; from ~48
    // columns (1.5 MiB per 1024-row tile) that stops working, and passes of
    // whole 256-byte row segments win: 2^20 x 184 172.6 -> 161.5 ms, 2^19 x 64
    // 27.8 -> 27.4 ms; at 8..32 columns the 2-pass plan stays ahead (2^19 x 14
    // 6.0 against 7.0 ms) -- tools/sweep_lde_logcw.sh, profiles/r02u_lde_logcw.txt
    static const int logcw_env = [] {
        const char* e = std::getenv("LSP_NTT_LOGCW");
        return e ? std::min(3, std::max(0, std::atoi(e))) : -1;
    }();
    static const bool twl_env = [] {  // LSP_NTT_TWL=0: the fused pass reads its twiddles from HBM
        const char* e = std::getenv("LSP_NTT_TWL");
        return !(e && *e == '0');
    }();
    static const uint32_t kmax_env = [] {
        const char* e = std::getenv("LSP_NTT_KMAX");
        return e ? (uint32_t)std::min(10, std::max(1, std::atoi(e))) : 10u;
    }();
    uint32_t logCWmax = 0;  // the power of two >= min(w, 8)
    while ((1u << logCWmax) < w && logCWmax < 3) ++logCWmax;
    const uint32_t logcw_min = logcw_env >= 0 ? (uint32_t)logcw_env : (w >= 48 ? 1u : 0u);
    const uint32_t kmax = std::min(kmax_env, 10 - std::min(logCWmax, logcw_min));
    uint32_t ks[16], np;
    plan_passes(logh, kmax, ks, np);
    // inverse: passes ks[0], ..., ks[np-1] (DIT, stages in increasing order);
    // forward: ks[np-1], ..., ks[0] (DIF), so the forward's first pass covers
    // the rows of the inverse's last pass and the two run as one (PASS_INV_FWD)
    auto launch = [&](bool dif, int mode, uint32_t k, uint32_t s0, uint32_t narr, const Fr* src, Fr* dst,
                      const uint4* tw, bool canon) -> hipError_t {
        // widest column chunk the 1024-element tile allows at this k (CW = 1 at k = 10)
        const uint32_t logCW = std::min(logCWmax, 10 - k);
        const uint32_t CW = 1u << logCW;
        const uint32_t nchunk = (uint32_t)((w + CW - 1) / CW);
        const uint32_t want = k + logCW >= 10 ? 0u : 10 - k - logCW;
        const uint32_t logG = std::min(logh - k, want);
        NttPass p;
        p.src = src;
        p.src_map = map;  // read only by the passes with a `src` (PASS_INV_FIRST / PASS_INV_FWD)
        p.no_inv = what == LDE_FWD ? 1u : 0u;
        p.dst = dst;
        p.tw = tw;
        p.tw_inv = tw_inv;
        p.inv_gather = (np == 1 && what == LDE_FULL) ? 1u : 0u;
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
        p.canon = canon ? 1u : 0u;
        p.narr = narr;
        p.ratio = mode == PASS_INV_FWD ? ratio : nullptr;
        p.log_narr = log_narr;
        // the fused pass loops over the cosets inside each workgroup
        const uint64_t tiles = (uint64_t)(mode == PASS_INV_FWD ? 1 : narr) * ((1ull << logh) >> (k + logG)) * nchunk;
        // tile, plus one twist (or chain ratio) factor per row in the fused pass
        const bool fac = mode == PASS_INV_FWD && (!twist_per_col || ratio);
        size_t lds = ((size_t(1) << (k + logG)) * CW + (fac ? (size_t(1) << (k + logG)) : 0)) * sizeof(F29);
        // ... and its forward twiddles when they fit (<= 512 entries, 18 KiB in planes: 2 workgroups per CU)
        const size_t twl_n = (size_t(1) << logG) * ((size_t(1) << k) - 1);
        p.twl_n = (mode == PASS_INV_FWD && twl_n <= 512 && twl_env) ? (uint32_t)twl_n : 0u;
        if (p.twl_n) lds = ((lds + 15) & ~(size_t)15) + (size_t)p.twl_n * TwlLds::BYTES;
        if (mode != PASS_INV_FWD) lds += (size_t)F29_QTAB_N * 3 * sizeof(uint4);  // k_ntt_rm's reduction table
        p.xcd = (tiles / nchunk) % 8 == 0 ? 1u : 0u;
        const dim3 grid((unsigned)tiles), blk(256);
#define LSP_NTT_LAUNCH(DIFV, MODEV)                                                                   \
    switch (logCW) {                                                                                  \
        case 0: hipLaunchKernelGGL((k_ntt_rm<DIFV, MODEV, 0>), grid, blk, lds, st, p); break;         \
        case 1: hipLaunchKernelGGL((k_ntt_rm<DIFV, MODEV, 1>), grid, blk, lds, st, p); break;         \
        case 2: hipLaunchKernelGGL((k_ntt_rm<DIFV, MODEV, 2>), grid, blk, lds, st, p); break;         \
        default: hipLaunchKernelGGL((k_ntt_rm<DIFV, MODEV, 3>), grid, blk, lds, st, p); break;        \
    }
        if (mode == PASS_INV_FWD) {
            LSP_NTT_LAUNCH(true, PASS_INV_FWD)
        } else if (dif) {
            LSP_NTT_LAUNCH(true, PASS_INPLACE)
        } else if (mode == PASS_INV_FIRST) {
            LSP_NTT_LAUNCH(false, PASS_INV_FIRST)
        } else {
            LSP_NTT_LAUNCH(false, PASS_INPLACE)
        }
#undef LSP_NTT_LAUNCH
        return hipGetLastError();
    };
    if (logh == 0) {
        // h = 1: the coefficient is the value; every coset row equals it
        if (what == LDE_INV || map.logb != COLMAP_PLAIN || map.c0 != 0 || map.cstep != 1 || map.stride != w)
            return hipErrorInvalidValue;  // (the sharded prover's maps never meet h = 1)
        for (uint32_t k = 0; k < ncosets; ++k) {
            hipError_t e = hipMemcpyAsync(out + (size_t)k * w, in, w * sizeof(Fr), hipMemcpyDeviceToDevice, st);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    hipError_t e = hipSuccess;
    if (what == LDE_INV) {  // every inverse pass, the last one too, into X
        uint32_t s0 = 0;
        for (uint32_t q = 0; q < np && e == hipSuccess; ++q) {
            e = launch(false, q == 0 ? PASS_INV_FIRST : PASS_INPLACE, ks[q], s0, 1, in, X, tw_inv, false);
            s0 += ks[q];
        }
        return e;
    }
    uint32_t s0 = 0;
    if (what == LDE_FULL)
        for (uint32_t q = 0; q + 1 < np; ++q) {  // inverse passes before the last
            e = launch(false, q == 0 ? PASS_INV_FIRST : PASS_INPLACE, ks[q], s0, 1, in, X, tw_inv, false);
            if (e != hipSuccess) return e;
            s0 += ks[q];
        }
    // the inverse's last stages (LDE_FULL) + the forward's first ks[np-1] stages, per coset
    e = launch(true, PASS_INV_FWD, ks[np - 1], 0, ncosets, (np == 1 || what == LDE_FWD) ? in : X, out, tw_fwd,
               np == 1);
    if (e != hipSuccess) return e;
    s0 = ks[np - 1];
    for (uint32_t q = 1; q < np; ++q) {  // the remaining forward passes
        const uint32_t k = ks[np - 1 - q];
        e = launch(true, PASS_INPLACE, k, s0, ncosets, out, out, tw_fwd, q + 1 == np);
        if (e != hipSuccess) return e;
        s0 += k;
    }
    return hipSuccess;
}

hipError_t launch_lde(const Fr* in, Fr* X, Fr* out, size_t w, uint32_t logh, uint32_t ncosets, const uint4* tw_inv,
                      const uint4* tw_fwd, const Fr* twist, uint32_t L1, uint32_t L2, int twist_per_col,
                      const Fr* ratio, hipStream_t st) {
    return run_lde(LDE_FULL, in, ColMap::plain((uint32_t)w), X, out, w, logh, ncosets, tw_inv, tw_fwd, twist, L1, L2,
                   twist_per_col, ratio, st);
}

hipError_t launch_intt(const Fr* in, ColMap map, Fr* X, size_t w, uint32_t logh, const uint4* tw_inv, hipStream_t st) {
    return run_lde(LDE_INV, in, map, X, nullptr, w, logh, 0, tw_inv, nullptr, nullptr, 0, 0, 0, nullptr, st);
}

hipError_t launch_lde_coeffs(const Fr* coef, ColMap map, Fr* out, size_t w, uint32_t logh, uint32_t ncosets,
                             const uint4* tw_fwd, const Fr* twist, uint32_t L1, uint32_t L2, int twist_per_col,
                             const Fr* ratio, hipStream_t st) {
    return run_lde(LDE_FWD, coef, map, nullptr, out, w, logh, ncosets, nullptr, tw_fwd, twist, L1, L2, twist_per_col,
                   ratio, st);
}

hipError_t launch_fold_subcoset(const Fr* coef, ColMap map, size_t h, size_t S, uint32_t w, const Fr* fac, Fr* out,
                                hipStream_t st) {
    if (S == 0 || h % S != 0 || h / S > 64 || w == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_fold_subcoset, dim3(nblocks(S * w, 256)), dim3(256), 0, st, coef, map, (uint64_t)h,
                       (uint64_t)S, w, (uint32_t)(h / S), fac, out);
    return hipGetLastError();
}

hipError_t launch_scale_coeffs(const Fr* X, size_t h, uint32_t w, const Fr* tab, uint32_t L1, Fr* out,
                               hipStream_t st) {
    if (h * w == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scale_coeffs, dim3(nblocks(h * w, 256)), dim3(256), 0, st, X, h, w, tab, L1, out);
    return hipGetLastError();
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

hipError_t launch_stage_twiddles(const Fr* pw, uint32_t logH, uint4* out, hipStream_t st) {
    const size_t n = (1ull << logH) - 1;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_stage_twiddles, dim3(nblocks(n, 256)), dim3(256), 0, st, pw, logH, out);
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

LSP_BOUNDS_READER(k_ntt)
