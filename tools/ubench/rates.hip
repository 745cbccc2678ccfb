// VALU instruction-rate probe on gfx950: cycles per wave64 instruction for
// v_mad_u64_u32, v_fma_f64, v_add_co/addc, v_mul_lo/hi_u32, v_fma_f32.
#include <hip/hip_runtime.h>
#include <cstdio>
#define N_IT 4096
template <int K> __global__ __launch_bounds__(256) void kr(unsigned long long* out, unsigned seed) {
    unsigned a = threadIdx.x + seed, b = a * 7 + 1;
    unsigned long long c0 = a, c1 = b, c2 = a ^ b, c3 = a + 9, c4 = a * 3, c5 = b * 5, c6 = a + b, c7 = b + 11;
    double d0 = a, d1 = b, d2 = a + 1.0, d3 = b + 2.0, d4 = a * 0.5, d5 = b * 0.25, d6 = 3.0, d7 = 5.0;
    float f0 = a, f1 = b, f2 = 1, f3 = 2, f4 = 3, f5 = 4, f6 = 5, f7 = 6;
    unsigned u0 = a, u1 = b, u2 = a + 1, u3 = b + 1, u4 = a + 2, u5 = b + 2, u6 = a + 3, u7 = b + 3;
    for (int i = 0; i < N_IT; ++i) {
        if (K == 0) {  // v_mad_u64_u32, 8 independent chains
#define M(c) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(c) : "v"(a), "v"(b) : "s40", "s41")
            M(c0); M(c1); M(c2); M(c3); M(c4); M(c5); M(c6); M(c7);
#undef M
        } else if (K == 1) {  // v_fma_f64
#define F(d) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d) : "v"(d6), "v"(d7))
            F(d0); F(d1); F(d2); F(d3); F(d4); F(d5); F(d6); F(d7);
#undef F
        } else if (K == 2) {  // v_add_co_u32 + v_addc_co_u32 pairs
#define A(x, y) asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc" : "+v"(x), "+v"(y) : "v"(a) : "vcc")
            A(u0, u1); A(u2, u3); A(u4, u5); A(u6, u7);
#undef A
        } else if (K == 3) {  // v_mul_hi_u32
#define H(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b))
            H(u0); H(u1); H(u2); H(u3); H(u4); H(u5); H(u6); H(u7);
#undef H
        } else if (K == 4) {  // v_fma_f32
#define G(x) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(f6), "v"(f7))
            G(f0); G(f1); G(f2); G(f3); G(f4); G(f5); G(f6); G(f7);
#undef G
        } else if (K == 5) {  // v_mul_lo_u32
#define L(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b))
            L(u0); L(u1); L(u2); L(u3); L(u4); L(u5); L(u6); L(u7);
#undef L
        } else if (K == 6) {  // v_lshl_add_u64 (64-bit add)
#define S(c) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(c) : "v"(c7))
            S(c0); S(c1); S(c2); S(c3); S(c4); S(c5); S(c6); S(c0);
#undef S
        } else if (K == 7) {  // v_add_f64
#define D(d) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d) : "v"(d7))
            D(d0); D(d1); D(d2); D(d3); D(d4); D(d5); D(d6); D(d0);
#undef D
        } else if (K == 8) {  // v_mad_u32_u24
#define U(x) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(x) : "v"(b))
            U(u0); U(u1); U(u2); U(u3); U(u4); U(u5); U(u6); U(u7);
#undef U
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7 + (unsigned long long)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7) +
        (unsigned long long)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7) + u0 + u1 + u2 + u3 + u4 + u5 + u6 + u7;
}
template <int K> void run(const char* nm, unsigned long long* out, int ninstr) {
    const int blocks = 256 * 8;  // 8 waves... 256 CUs x 2 blocks of 4 waves
    hipLaunchKernelGGL(kr<K>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kr<K>, dim3(blocks), dim3(256), 0, 0, out, 2u);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    double waves = blocks * 256.0 / 64, instr = waves * N_IT * ninstr;
    double per_simd_cycles = ms * 1e-3 * 2.4e9 * 1024;  // SIMD-cycles available
    printf("%-22s %8.3f ms  %6.2f cycles per wave64 instruction per SIMD (at 2.4 GHz)\n", nm, ms, per_simd_cycles / instr);
}
int main() {
    unsigned long long* out; (void)hipMalloc(&out, 256 * 8 * 256 * 8);
    run<0>("v_mad_u64_u32", out, 8);
    run<1>("v_fma_f64", out, 8);
    run<2>("v_add_co+addc (x2)", out, 8);
    run<3>("v_mul_hi_u32", out, 8);
    run<4>("v_fma_f32", out, 8);
    run<5>("v_mul_lo_u32", out, 8);
    run<6>("v_lshl_add_u64", out, 8);
    run<7>("v_add_f64", out, 8);
    run<8>("v_mad_u32_u24", out, 8);
    return 0;
}
