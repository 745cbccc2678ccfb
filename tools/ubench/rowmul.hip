// A limb-parallel Fr product for the narrow Merkle levels,
// measured instead of estimated: one 29-bit-limb Montgomery product (the same
// function as f29_mul, fr29.hpp) spread over a 16-lane DPP row -- lane l of
// the row holds limb l (0 beyond 8) -- so one wave computes four products,
// one per row.  Product scanning: column k accumulates in lane k, a_j reaches
// every lane by `row_newbcast:j`, b moves one lane per step by `row_shr:1`;
// REDC digit by digit, the column's 64-bit sum broadcast to the row, the digit
// and carry computed in every lane, the digit's multiple of r added to the
// columns by one MAD per step; then the output columns 9..16 normalised with a
// carry chain and selected into lanes 0..8.
//
// Times one wave (64 lanes = 4 rows) alone on the chip, as tools/ubench/
// latbench.hip does for f29_mul: cycles per dependent product (s_memtime),
// and checks every row's result against f29_mul_c of the same operands.
//   build: tools/ubench/build.sh rowmul    run: tools/ubench/rowmul
#include <cstdio>
#include <cstdint>
#include <hip/hip_runtime.h>
#include "../../linea_stark_prover_amd/csrc/fr29.hpp"
using namespace lsp;
namespace lsp {
#include "../../linea_stark_prover_amd/csrc/fr29_row_gfx950.inc"
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t bcast(uint32_t x, int n) {  // lane n of this lane's row
    switch (n) {
        case 0: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150, 0xf, 0xf, false);
        case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x151, 0xf, 0xf, false);
        case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x152, 0xf, 0xf, false);
        case 3: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x153, 0xf, 0xf, false);
        case 4: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x154, 0xf, 0xf, false);
        case 5: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x155, 0xf, 0xf, false);
        case 6: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x156, 0xf, 0xf, false);
        case 7: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x157, 0xf, 0xf, false);
        case 8: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x158, 0xf, 0xf, false);
        case 9: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x159, 0xf, 0xf, false);
        case 10: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x15a, 0xf, 0xf, false);
        case 11: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x15b, 0xf, 0xf, false);
        case 12: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x15c, 0xf, 0xf, false);
        case 13: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x15d, 0xf, 0xf, false);
        case 14: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x15e, 0xf, 0xf, false);
        default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x15f, 0xf, 0xf, false);
    }
}
__device__ __forceinline__ uint32_t shr1(uint32_t x) {  // lane l <- lane l - 1 of the row, lane 0 <- 0
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xf, 0xf, true);
}
__device__ __forceinline__ uint64_t bcast64(uint64_t x, int n) {
    return (uint64_t)bcast((uint32_t)x, n) | ((uint64_t)bcast((uint32_t)(x >> 32), n) << 32);
}

// per-lane constants: c29(l) for l <= 8; P[k] = p29(l - k) for 1 <= l - k <= 8
struct RowConst {
    uint32_t c;
    uint32_t P[9];
};
__device__ __forceinline__ RowConst row_const(uint32_t l) {
    RowConst k;
    k.c = l <= 8 ? c29((int)l) : 0u;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        const int d = (int)l - j;
        k.P[j] = (d >= 1 && d <= 8) ? p29(d) : 0u;
    }
    return k;
}

// a, b: this lane's limb (lane % 16 = limb index, 0 beyond 8); returns the
// product's limb for this lane (0 beyond 8)
__device__ __forceinline__ uint32_t rowmul(uint32_t a, uint32_t b, const RowConst& K, uint32_t l) {
    uint64_t acc = K.c;
    uint32_t bs = b;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        acc += (uint64_t)bcast(a, j) * bs;
        bs = shr1(bs);
    }
    uint64_t col16 = (uint64_t)bcast(a, 8) * bcast(b, 8);
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const uint64_t v = bcast64(acc, k) + carry;
        const uint32_t m = ~(uint32_t)v;
        carry = (v >> 32) * 8 + 7;
        acc += (uint64_t)m * K.P[k];
        if (k == 8) col16 += (uint64_t)m * p29(8);
    }
    uint32_t out = 0;
#pragma unroll
    for (int c = 9; c <= 16; ++c) {
        const uint64_t v = (c < 16 ? bcast64(acc, c) : col16) + carry;
        out = l == (uint32_t)(c - 9) ? ((uint32_t)v & F29_MASK) : out;
        carry = v >> 29;
    }
    return l == 8 ? (uint32_t)carry : out;
}

__device__ __forceinline__ uint32_t shl9(uint32_t x) {  // lane l <- lane l + 9 of the row, beyond -> 0
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x109, 0xf, 0xf, true);
}

// The same product with the output columns normalised in parallel instead of
// by a carry chain across lanes: the columns move down to lanes 0..7 (row_shl:9),
// then carry-save rounds (limb & mask + the lane below's limb >> 29, via
// row_shr:1) until no carry is left -- three rounds reach limbs <= 2^29 for any
// column sums below 2^64 (enough for this measurement: a product operand may
// exceed 2^29 - 1 by one, which fr29.hpp's bounds would have to admit).
__device__ __forceinline__ uint32_t rowmul2(uint32_t a, uint32_t b, const RowConst& K, uint32_t l) {
    uint64_t acc = K.c;
    uint32_t bs = b;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        acc += (uint64_t)bcast(a, j) * bs;
        bs = shr1(bs);
    }
    uint64_t col16 = (uint64_t)bcast(a, 8) * bcast(b, 8);
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const uint64_t v = bcast64(acc, k) + carry;
        const uint32_t m = ~(uint32_t)v;
        carry = (v >> 32) * 8 + 7;
        acc += (uint64_t)m * K.P[k];
        if (k == 8) col16 += (uint64_t)m * p29(8);
    }
    // columns 9..15 -> lanes 0..6, column 16 -> lane 7, the pending carry into lane 0
    uint64_t x = (uint64_t)shl9((uint32_t)acc) | ((uint64_t)shl9((uint32_t)(acc >> 32)) << 32);
    x = l == 7 ? col16 : x;
    x += l == 0 ? carry : 0;
    // round 1: 64-bit carries (< 2^35)
    uint64_t c = x >> 29;
    uint32_t lo = (uint32_t)x & F29_MASK;
    uint64_t cs = (uint64_t)shr1((uint32_t)c) | ((uint64_t)shr1((uint32_t)(c >> 32)) << 32);
    uint64_t y = lo + cs;  // < 2^29 + 2^35; lane 8 receives lane 7's carry (the top limb)
    // rounds 2, 3: 32-bit carries
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const uint32_t cc = (uint32_t)(y >> 29);
        const uint32_t keep = l == 8 ? 0xffffffffu : F29_MASK;  // the top limb keeps its bits
        y = ((uint32_t)y & keep) + (l == 8 ? 0u : 0u) + shr1(l == 8 ? 0u : cc);
    }
    return l <= 8 ? (uint32_t)y : 0u;
}

template <int V>
__global__ void krow(uint32_t* out, uint64_t* cyc, int iters, uint32_t* check) {
    const uint32_t lane = threadIdx.x & 63, l = lane & 15, row = lane >> 4;
    const RowConst K = row_const(l);
    // operands: row r's a = f29_from_fr(r + 3), m = f29_from_fr(0x1234567 + r), limb l on lane l
    const F29 A = f29_from_fr(fr_from_u64(row + 3)), M = f29_from_fr(fr_from_u64(0x1234567 + row));
    uint32_t a = 0, m = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        a = l == (uint32_t)i ? A.l[i] : a;
        m = l == (uint32_t)i ? M.l[i] : m;
    }
    // correctness: one product against f29_mul_c
    const F29RowK KA = f29row_consts(l);
    auto mulv = [&](uint32_t x, uint32_t y) { return V == 1 ? rowmul(x, y, K, l) : V == 2 ? rowmul2(x, y, K, l) : f29row_mul(x, y, KA); };
    const uint32_t p1 = mulv(a, m);
    const F29 ref = f29_mul_c(A, M);
    uint32_t want = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) want = l == (uint32_t)i ? ref.l[i] : want;
    // carry-save outputs may leave a limb at 2^29: compare the values (the row's
    // limbs gathered and carried) and that lanes 9..15 hold zero
    uint32_t bad = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        F29 g;
        for (int i = 0; i < 9; ++i) g.l[i] = __builtin_amdgcn_readlane(p1, r * 16 + i);
        uint64_t cy = 0;
        for (int i = 0; i < 9; ++i) {
            const uint64_t v = (uint64_t)g.l[i] + cy;
            g.l[i] = i < 8 ? (uint32_t)v & F29_MASK : (uint32_t)v;
            cy = v >> 29;
        }
        if (r == (int)row && l < 9 && g.l[l] != want) bad = 1;
    }
    if (l >= 9 && p1 != 0) bad = 1;
    check[threadIdx.x] = bad;
    const uint64_t t0 = clock64();
    for (int i = 0; i < iters; ++i) a = mulv(a, m);
    const uint64_t t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void kf29(Fr* out, uint64_t* cyc, int iters) {
    F29 a = f29_from_fr(fr_from_u64(threadIdx.x + 3));
    const F29 m = f29_from_fr(fr_from_u64(0x1234567 + threadIdx.x));
    const uint64_t t0 = clock64();
    for (int i = 0; i < iters; ++i) a = f29_mul(a, m);
    const uint64_t t1 = clock64();
    out[threadIdx.x] = f29_to_fr(a);
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    uint32_t *out, *chk;
    uint64_t* cyc;
    Fr* fo;
    CK(hipMalloc(&out, 64 * 4)); CK(hipMalloc(&chk, 64 * 4)); CK(hipMalloc(&cyc, 8)); CK(hipMalloc(&fo, 64 * sizeof(Fr)));
    const int it = 2000;
    uint64_t c;
    uint32_t h[64];
    for (int rep = 0; rep < 3; ++rep) {
        double row[3];
        int bad[3];
        for (int v = 0; v < 3; ++v) {
            if (v == 0) hipLaunchKernelGGL(krow<1>, dim3(1), dim3(64), 0, 0, out, cyc, it, chk);
            else if (v == 1) hipLaunchKernelGGL(krow<2>, dim3(1), dim3(64), 0, 0, out, cyc, it, chk);
            else hipLaunchKernelGGL(krow<3>, dim3(1), dim3(64), 0, 0, out, cyc, it, chk);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(h, chk, sizeof h, hipMemcpyDeviceToHost));
            bad[v] = 0;
            for (int i = 0; i < 64; ++i) bad[v] += h[i];
            row[v] = (double)c / it;
        }
        hipLaunchKernelGGL(kf29, dim3(1), dim3(64), 0, 0, fo, cyc, it);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
        const double lane = (double)c / it;
        printf("one wave alone, cycles per dependent product: f29_mul (one lane per product) %.1f; row product "
               "(16 lanes per product, compiled) %.1f (%.2fx), with carry-save output %.1f (%.2fx), hand-scheduled "
               "asm (fr29_row_gfx950.inc) %.1f (%.2fx); mismatches %d / %d / %d\n",
               lane, row[0], lane / row[0], row[1], lane / row[1], row[2], lane / row[2], bad[0], bad[1], bad[2]);
    }
    return 0;
}
