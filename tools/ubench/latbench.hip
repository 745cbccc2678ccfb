// Single-wave issue latency of v_mad_u64_u32: one wave alone on the chip runs
// a loop of 64 MADs as 1, 2, 4 or 8 independent accumulator chains, timed with
// s_memtime (shader clock) around the loop.  Tells whether a lone wave (the
// narrow Merkle levels: one or fewer waves per SIMD) is bound by the MAD's
// dependent latency -- then a product with several accumulator chains would
// run faster there -- or by its issue interval.  Also the shipped 29-bit
// product as a dependent chain (f29_mul) for reference.
//   build: tools/ubench/build.sh latbench    run: tools/ubench/latbench
#include <cstdio>
#include <cstdint>
#include <hip/hip_runtime.h>
#include "../../linea_stark_prover_amd/csrc/fr29.hpp"
using namespace lsp;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define MAD1(acc) "v_mad_u64_u32 " acc ", %[c], %[x], %[y], " acc "\n\t"

template <int C>
__global__ void kmad(uint64_t* out, uint64_t* cyc, int iters) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, c;
    const uint32_t x = 0x1234567u + threadIdx.x, y = 0x7654321u;
    const uint64_t t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        if constexpr (C == 1) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                asm volatile(MAD1("%[a0]") MAD1("%[a0]") MAD1("%[a0]") MAD1("%[a0]") MAD1("%[a0]") MAD1("%[a0]")
                             MAD1("%[a0]") MAD1("%[a0]")
                             : [a0] "+v"(a0), [c] "=s"(c) : [x] "v"(x), [y] "v"(y));
        } else if constexpr (C == 2) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                asm volatile(MAD1("%[a0]") MAD1("%[a1]") MAD1("%[a0]") MAD1("%[a1]") MAD1("%[a0]") MAD1("%[a1]")
                             MAD1("%[a0]") MAD1("%[a1]")
                             : [a0] "+v"(a0), [a1] "+v"(a1), [c] "=s"(c) : [x] "v"(x), [y] "v"(y));
        } else if constexpr (C == 4) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                asm volatile(MAD1("%[a0]") MAD1("%[a1]") MAD1("%[a2]") MAD1("%[a3]") MAD1("%[a0]") MAD1("%[a1]")
                             MAD1("%[a2]") MAD1("%[a3]")
                             : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [c] "=s"(c)
                             : [x] "v"(x), [y] "v"(y));
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                asm volatile(MAD1("%[a0]") MAD1("%[a1]") MAD1("%[a2]") MAD1("%[a3]") MAD1("%[a4]") MAD1("%[a5]")
                             MAD1("%[a6]") MAD1("%[a7]")
                             : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [a4] "+v"(a4),
                               [a5] "+v"(a5), [a6] "+v"(a6), [a7] "+v"(a7), [c] "=s"(c)
                             : [x] "v"(x), [y] "v"(y));
        }
    }
    const uint64_t t1 = clock64();
    out[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// 32-bit adds: a dependent chain vs 4 independent (the 2-cycle class)
template <int C>
__global__ void kadd(uint32_t* out, uint64_t* cyc, int iters) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    const uint32_t x = 0x1234567u + threadIdx.x;
    const uint64_t t0 = clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (C == 1)
                asm volatile("v_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\t"
                             "v_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1"
                             : "+v"(a0) : "v"(x));
            else
                asm volatile("v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4\n\t"
                             "v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x));
        }
    }
    const uint64_t t1 = clock64();
    out[threadIdx.x] = a0 + a1 + a2 + a3;
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

__global__ void kf29x2(Fr* out, uint64_t* cyc, int iters) {
    F29 a = f29_from_fr(fr_from_u64(threadIdx.x + 3)), b = f29_from_fr(fr_from_u64(threadIdx.x + 5));
    const F29 m = f29_from_fr(fr_from_u64(0x1234567 + threadIdx.x));
    const uint64_t t0 = clock64();
    for (int i = 0; i < iters; ++i) { a = f29_mul(a, m); b = f29_mul(b, m); }
    const uint64_t t1 = clock64();
    out[threadIdx.x] = fr_add(f29_to_fr(a), f29_to_fr(b));
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    uint64_t *out, *cyc;
    Fr* fo;
    CK(hipMalloc(&out, 64 * 8)); CK(hipMalloc(&cyc, 8)); CK(hipMalloc(&fo, 64 * sizeof(Fr)));
    const int it = 2000;
    uint64_t c;
    auto rd = [&]() { (void)hipDeviceSynchronize(); (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost); return (double)c; };
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(kmad<1>, dim3(1), dim3(64), 0, 0, out, cyc, it); double c1 = rd();
        hipLaunchKernelGGL(kmad<2>, dim3(1), dim3(64), 0, 0, out, cyc, it); double c2 = rd();
        hipLaunchKernelGGL(kmad<4>, dim3(1), dim3(64), 0, 0, out, cyc, it); double c4 = rd();
        hipLaunchKernelGGL(kmad<8>, dim3(1), dim3(64), 0, 0, out, cyc, it); double c8 = rd();
        const double n = 64.0 * it;
        printf("v_mad_u64_u32, one wave: cycles per MAD with 1 / 2 / 4 / 8 chains: %.2f %.2f %.2f %.2f\n", c1 / n, c2 / n,
               c4 / n, c8 / n);
        hipLaunchKernelGGL(kadd<1>, dim3(1), dim3(64), 0, 0, (uint32_t*)out, cyc, it); double d1 = rd();
        hipLaunchKernelGGL(kadd<4>, dim3(1), dim3(64), 0, 0, (uint32_t*)out, cyc, it); double d4 = rd();
        printf("v_add_u32, one wave: cycles per add with 1 / 4 chains: %.2f %.2f\n", d1 / n, d4 / n);
        hipLaunchKernelGGL(kf29, dim3(1), dim3(64), 0, 0, fo, cyc, it); double f1 = rd();
        hipLaunchKernelGGL(kf29x2, dim3(1), dim3(64), 0, 0, fo, cyc, it); double f2 = rd();
        printf("f29_mul, one wave: cycles per product, dependent chain %.1f; two independent chains %.1f per product\n",
               f1 / it, f2 / (2.0 * it));
    }
    return 0;
}
