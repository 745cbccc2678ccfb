// VALU instruction-rate probe for gfx950 (MI355X): cycles per wave64
// instruction per SIMD, measured in shader clock cycles (s_memtime) inside
// the kernel, at 1, 2, 4 and 8 resident waves per SIMD.
//
//   hipcc --offload-arch=gfx950 -O3 -o rates rates.hip && ./rates [--json out.json]
//
// Every instruction class runs 8 independent dependency chains per wave, so
// with >= 2 waves per SIMD the figure is the issue throughput, and at one wave
// it is the issue cost of one wave's stream.  Grid = 256 CUs x 4 SIMDs x W
// waves (256-thread blocks of 4 waves), so each SIMD holds W waves at once; the
// per-wave elapsed cycles (median over waves) divided by (instructions x W) is
// the SIMD's cycles per wave64 instruction.  s_memrealtime (100 MHz) gives the
// clock the chip held during the run.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#define N_IT 8192

struct Sample { unsigned long long cyc, rt, rt0, rt1; };

// K selects the instruction class; each iteration issues 8 instructions.
template <int K> __global__ __launch_bounds__(256) void kr(Sample* out, unsigned long long* sink, unsigned seed) {
    unsigned a = threadIdx.x + seed, b = a * 7 + 1;
    unsigned long long c0 = a, c1 = b, c2 = a ^ b, c3 = a + 9, c4 = a * 3, c5 = b * 5, c6 = a + b, c7 = b + 11;
    double d0 = a, d1 = b, d2 = a + 1.0, d3 = b + 2.0, d4 = a * 0.5, d5 = b * 0.25, d6 = 3.0, d7 = 5.0;
    const double dk0 = 1.0000001, dk1 = 0.9999999;
    float f0 = a, f1 = b, f2 = 1, f3 = 2, f4 = 3, f5 = 4, f6 = 5, f7 = 6;
    const float fa = 1.0001f, fb = 0.9999f;
    unsigned u0 = a, u1 = b, u2 = a + 1, u3 = b + 1, u4 = a + 2, u5 = b + 2, u6 = a + 3, u7 = b + 3;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < N_IT; ++i) {
        if (K == 0) {  // v_mad_u64_u32 (carry-out to an SGPR pair)
#define M(c) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(c) : "v"(a), "v"(b) : "s40", "s41")
            M(c0); M(c1); M(c2); M(c3); M(c4); M(c5); M(c6); M(c7);
#undef M
        } else if (K == 1) {  // v_fma_f64
#define F(d) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d) : "v"(dk0), "v"(dk1))
            F(d0); F(d1); F(d2); F(d3); F(d4); F(d5); F(d6); F(d7);
#undef F
        } else if (K == 2) {  // v_add_co_u32 / v_addc_co_u32 pairs (8 instructions)
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
#define D(d) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d) : "v"(dk1))
            D(d0); D(d1); D(d2); D(d3); D(d4); D(d5); D(d6); D(d7);
#undef D
        } else if (K == 8) {  // v_mad_u32_u24
#define U(x) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(x) : "v"(b))
            U(u0); U(u1); U(u2); U(u3); U(u4); U(u5); U(u6); U(u7);
#undef U
        } else if (K == 9) {  // v_lshrrev_b64
#define R(c) asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(c))
            R(c0); R(c1); R(c2); R(c3); R(c4); R(c5); R(c6); R(c7);
#undef R
        } else if (K == 10) {  // v_add_u32
#define P(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b))
            P(u0); P(u1); P(u2); P(u3); P(u4); P(u5); P(u6); P(u7);
#undef P
        } else if (K == 11) {  // v_and_b32
#define N(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(b))
            N(u0); N(u1); N(u2); N(u3); N(u4); N(u5); N(u6); N(u7);
#undef N
        } else if (K == 12) {  // v_mul_f64
#define Q(d) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d) : "v"(dk0))
            Q(d0); Q(d1); Q(d2); Q(d3); Q(d4); Q(d5); Q(d6); Q(d7);
#undef Q
        } else if (K == 13) {  // v_pk_fma_f32 (2 FP32 FMAs per lane)
#define PK(x) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(dk0), "v"(dk1))
            PK(d0); PK(d1); PK(d2); PK(d3); PK(d4); PK(d5); PK(d6); PK(d7);
#undef PK
        } else if (K == 14) {  // v_add3_u32
#define T3(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b))
            T3(u0); T3(u1); T3(u2); T3(u3); T3(u4); T3(u5); T3(u6); T3(u7);
#undef T3
        } else if (K == 15) {  // v_alignbit_b32 (funnel shift)
#define AB(x, y) asm volatile("v_alignbit_b32 %0, %1, %0, 29" : "+v"(x) : "v"(y))
            AB(u0, u1); AB(u1, u2); AB(u2, u3); AB(u3, u4); AB(u4, u5); AB(u5, u6); AB(u6, u7); AB(u7, u0);
#undef AB
        } else if (K == 16) {  // v_mov_b32 with DPP quad_perm (cross-lane)
#define DP(x, y) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(x) : "v"(y))
            DP(u0, u1); DP(u1, u2); DP(u2, u3); DP(u3, u4); DP(u4, u5); DP(u5, u6); DP(u6, u7); DP(u7, u0);
#undef DP
        } else if (K == 18) {  // v_add_u32 in the VOP3 encoding
#define P3(x) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(b))
            P3(u0); P3(u1); P3(u2); P3(u3); P3(u4); P3(u5); P3(u6); P3(u7);
#undef P3
        } else if (K == 19) {  // v_lshlrev_b32 (VOP2)
#define SL(x) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x))
            SL(u0); SL(u1); SL(u2); SL(u3); SL(u4); SL(u5); SL(u6); SL(u7);
#undef SL
        } else if (K == 20) {  // v_not_b32 (VOP1)
#define NT(x) asm volatile("v_not_b32 %0, %0" : "+v"(x))
            NT(u0); NT(u1); NT(u2); NT(u3); NT(u4); NT(u5); NT(u6); NT(u7);
#undef NT
        } else if (K == 21) {  // v_lshl_or_b32 (VOP3, 3 sources)
#define LO(x) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x) : "v"(b))
            LO(u0); LO(u1); LO(u2); LO(u3); LO(u4); LO(u5); LO(u6); LO(u7);
#undef LO
        } else if (K == 22) {  // v_fma_f32 with loop-invariant multiplicands
#define G2(x) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(fa), "v"(fb))
            G2(f0); G2(f1); G2(f2); G2(f3); G2(f4); G2(f5); G2(f6); G2(f7);
#undef G2
        } else if (K == 23) {  // v_mad_u64_u32 and v_add_u32 interleaved (4 + 4)
#define MI(c, x) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %3, %0\n\tv_add_u32 %1, %1, %3" : "+v"(c), "+v"(x) : "v"(a), "v"(b) : "s40", "s41")
            MI(c0, u0); MI(c1, u1); MI(c2, u2); MI(c3, u3);
#undef MI
        } else if (K == 24) {  // v_bfe_u32 (VOP3)
#define BF(x) asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(x))
            BF(u0); BF(u1); BF(u2); BF(u3); BF(u4); BF(u5); BF(u6); BF(u7);
#undef BF
        } else if (K == 25) {  // v_mad_u64_u32 with an inline-constant multiplicand
#define MC(c) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, 1, %0" : "+v"(c) : "v"(a) : "s40", "s41")
            MC(c0); MC(c1); MC(c2); MC(c3); MC(c4); MC(c5); MC(c6); MC(c7);
#undef MC
        } else if (K == 26) {  // v_lshrrev_b32 (VOP2)
#define SR(x) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(x))
            SR(u0); SR(u1); SR(u2); SR(u3); SR(u4); SR(u5); SR(u6); SR(u7);
#undef SR
        } else if (K == 27) {  // v_mad_u64_u32 with an SGPR multiplicand
#define MS(c) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(c) : "v"(a), "s"(seed) : "s40", "s41")
            MS(c0); MS(c1); MS(c2); MS(c3); MS(c4); MS(c5); MS(c6); MS(c7);
#undef MS
        } else if (K == 28) {  // v_mad_u64_u32 and v_fma_f64 interleaved: separate pipes?
#define MF(c, dd) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %3, %0\n\tv_fma_f64 %1, %4, %5, %1" : "+v"(c), "+v"(dd) : "v"(a), "v"(b), "v"(dk0), "v"(dk1) : "s40", "s41")
            MF(c0, d0); MF(c1, d1); MF(c2, d2); MF(c3, d3);
#undef MF
        } else if (K == 29) {  // v_mad_u64_u32 and v_pk_fma_f32 interleaved
#define MP(c, dd) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %3, %0\n\tv_pk_fma_f32 %1, %4, %5, %1" : "+v"(c), "+v"(dd) : "v"(a), "v"(b), "v"(dk0), "v"(dk1) : "s40", "s41")
            MP(c0, d0); MP(c1, d1); MP(c2, d2); MP(c3, d3);
#undef MP
        } else if (K == 30) {  // v_mad_u64_u32 and v_mad_u32_u24 interleaved
#define M24(c, x) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %3, %0\n\tv_mad_u32_u24 %1, %1, %3, %1" : "+v"(c), "+v"(x) : "v"(a), "v"(b) : "s40", "s41")
            M24(c0, u0); M24(c1, u1); M24(c2, u2); M24(c3, u3);
#undef M24
        } else if (K == 31) {  // v_mad_u64_u32 and v_lshrrev_b64 interleaved
#define ML(c, cc) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %3, %0\n\tv_lshrrev_b64 %1, 29, %1" : "+v"(c), "+v"(cc) : "v"(a), "v"(b) : "s40", "s41")
            ML(c0, c4); ML(c1, c5); ML(c2, c6); ML(c3, c7);
#undef ML
        } else if (K == 32) {  // v_fma_f64 and v_add_u32 interleaved
#define FA(dd, x) asm volatile("v_fma_f64 %0, %2, %3, %0\n\tv_add_u32 %1, %1, %4" : "+v"(dd), "+v"(x) : "v"(dk0), "v"(dk1), "v"(b))
            FA(d0, u0); FA(d1, u1); FA(d2, u2); FA(d3, u3);
#undef FA
        } else if (K == 33) {  // v_mul_hi_u32 and v_mul_lo_u32 interleaved (32-bit multiplier)
#define HL(x, y) asm volatile("v_mul_hi_u32 %0, %0, %2\n\tv_mul_lo_u32 %1, %1, %2" : "+v"(x), "+v"(y) : "v"(b))
            HL(u0, u1); HL(u2, u3); HL(u4, u5); HL(u6, u7);
#undef HL
        } else if (K == 34) {  // v_mad_i64_i32 (signed; the signed-digit product)
#define MSI(c) asm volatile("v_mad_i64_i32 %0, s[40:41], %1, %2, %0" : "+v"(c) : "v"(a), "v"(b) : "s40", "s41")
            MSI(c0); MSI(c1); MSI(c2); MSI(c3); MSI(c4); MSI(c5); MSI(c6); MSI(c7);
#undef MSI
        } else if (K == 35) {  // v_ashrrev_i64 (the signed carries)
#define AS(c) asm volatile("v_ashrrev_i64 %0, 29, %0" : "+v"(c))
            AS(c0); AS(c1); AS(c2); AS(c3); AS(c4); AS(c5); AS(c6); AS(c7);
#undef AS
        } else if (K == 17) {  // v_sub_u32 chains on a 64-bit pair: v_sub_co_u32 / v_subb_co_u32 (8 instructions)
#define SB(x, y) asm volatile("v_sub_co_u32 %0, vcc, %0, %2\n\tv_subb_co_u32 %1, vcc, %1, %2, vcc" : "+v"(x), "+v"(y) : "v"(a) : "vcc")
            SB(u0, u1); SB(u2, u3); SB(u4, u5); SB(u6, u7);
#undef SB
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = Sample{t1 - t0, r1 - r0, r0, r1};
    sink[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7 +
        (unsigned long long)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7) +
        (unsigned long long)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7) + u0 + u1 + u2 + u3 + u4 + u5 + u6 + u7;
}

struct Row { std::string name; double cyc[4]; double ghz[4]; double span[4]; };

template <int K> Row run(const char* nm, Sample* out, unsigned long long* sink, int cus) {
    Row row{nm, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    const int Ws[4] = {1, 2, 4, 8};
    for (int wi = 0; wi < 4; ++wi) {
        int W = Ws[wi];
        int blocks = cus * W;  // 256-thread blocks = 4 waves = one per SIMD of a CU
        hipLaunchKernelGGL(kr<K>, dim3(blocks), dim3(256), 0, 0, out, sink, 1u);  // warm
        hipLaunchKernelGGL(kr<K>, dim3(blocks), dim3(256), 0, 0, out, sink, 2u);
        (void)hipDeviceSynchronize();
        int nw = blocks * 4;
        std::vector<Sample> s(nw);
        (void)hipMemcpy(s.data(), out, nw * sizeof(Sample), hipMemcpyDeviceToHost);
        std::vector<double> c(nw), g(nw);
        for (int i = 0; i < nw; ++i) { c[i] = (double)s[i].cyc; g[i] = s[i].rt ? s[i].cyc / (s[i].rt * 10.0) : 0; }
        std::sort(c.begin(), c.end());
        std::sort(g.begin(), g.end());
        row.cyc[wi] = c[nw / 2] / ((double)N_IT * 8 * W);
        row.ghz[wi] = g[nw / 2];
        unsigned long long lo = ~0ull, hi = 0;
        for (auto& x : s) { lo = std::min(lo, x.rt0); hi = std::max(hi, x.rt1); }
        // whole-grid span: first wave's start to last wave's end (100 MHz), at the median clock
        const double span_cyc = (hi - lo) * 10.0 * g[nw / 2];
        row.span[wi] = span_cyc * (cus * 4.0) / ((double)nw * N_IT * 8);
    }
    return row;
}

int main(int argc, char** argv) {
    const char* json = nullptr;
    for (int i = 1; i < argc; ++i)
        if (!strcmp(argv[i], "--json") && i + 1 < argc) json = argv[++i];
    hipDeviceProp_t pr;
    (void)hipGetDeviceProperties(&pr, 0);
    int cus = pr.multiProcessorCount;
    Sample* out;
    unsigned long long* sink;
    (void)hipMalloc(&out, (size_t)cus * 8 * 4 * sizeof(Sample));
    (void)hipMalloc(&sink, (size_t)cus * 8 * 256 * 8);
    std::vector<Row> rows;
    rows.push_back(run<0>("v_mad_u64_u32", out, sink, cus));
    rows.push_back(run<1>("v_fma_f64", out, sink, cus));
    rows.push_back(run<12>("v_mul_f64", out, sink, cus));
    rows.push_back(run<7>("v_add_f64", out, sink, cus));
    rows.push_back(run<13>("v_pk_fma_f32", out, sink, cus));
    rows.push_back(run<4>("v_fma_f32", out, sink, cus));
    rows.push_back(run<2>("v_add_co_u32+v_addc_co_u32", out, sink, cus));
    rows.push_back(run<17>("v_sub_co_u32+v_subb_co_u32", out, sink, cus));
    rows.push_back(run<10>("v_add_u32", out, sink, cus));
    rows.push_back(run<14>("v_add3_u32", out, sink, cus));
    rows.push_back(run<11>("v_and_b32", out, sink, cus));
    rows.push_back(run<15>("v_alignbit_b32", out, sink, cus));
    rows.push_back(run<9>("v_lshrrev_b64", out, sink, cus));
    rows.push_back(run<6>("v_lshl_add_u64", out, sink, cus));
    rows.push_back(run<3>("v_mul_hi_u32", out, sink, cus));
    rows.push_back(run<5>("v_mul_lo_u32", out, sink, cus));
    rows.push_back(run<8>("v_mad_u32_u24", out, sink, cus));
    rows.push_back(run<16>("v_mov_b32_dpp quad_perm", out, sink, cus));
    rows.push_back(run<18>("v_add_u32_e64 (VOP3)", out, sink, cus));
    rows.push_back(run<19>("v_lshlrev_b32", out, sink, cus));
    rows.push_back(run<26>("v_lshrrev_b32", out, sink, cus));
    rows.push_back(run<20>("v_not_b32", out, sink, cus));
    rows.push_back(run<21>("v_lshl_or_b32", out, sink, cus));
    rows.push_back(run<24>("v_bfe_u32", out, sink, cus));
    rows.push_back(run<22>("v_fma_f32 (invariant operands)", out, sink, cus));
    rows.push_back(run<23>("v_mad_u64_u32 + v_add_u32 (1:1)", out, sink, cus));
    rows.push_back(run<25>("v_mad_u64_u32 (x inline 1)", out, sink, cus));
    rows.push_back(run<27>("v_mad_u64_u32 (x SGPR)", out, sink, cus));
    rows.push_back(run<28>("v_mad_u64_u32 + v_fma_f64 (1:1)", out, sink, cus));
    rows.push_back(run<29>("v_mad_u64_u32 + v_pk_fma_f32 (1:1)", out, sink, cus));
    rows.push_back(run<30>("v_mad_u64_u32 + v_mad_u32_u24 (1:1)", out, sink, cus));
    rows.push_back(run<31>("v_mad_u64_u32 + v_lshrrev_b64 (1:1)", out, sink, cus));
    rows.push_back(run<32>("v_fma_f64 + v_add_u32 (1:1)", out, sink, cus));
    rows.push_back(run<33>("v_mul_hi_u32 + v_mul_lo_u32 (1:1)", out, sink, cus));
    rows.push_back(run<34>("v_mad_i64_i32", out, sink, cus));
    rows.push_back(run<35>("v_ashrrev_i64", out, sink, cus));
    printf("device %s, %d CUs; cycles per wave64 instruction per SIMD (shader clock, s_memtime), "
           "median over waves; GHz = s_memtime / s_memrealtime\n", pr.gcnArchName, cus);
    printf("%-34s %21s   %27s   %s\n", "", "per-wave median", "whole-grid span", "");
    printf("%-34s %6s %6s %6s %6s   %6s %6s %6s %6s   %s\n", "instruction", "W=1", "W=2", "W=4", "W=8", "W=1", "W=2",
           "W=4", "W=8", "GHz(W=1..8)");
    for (auto& r : rows)
        printf("%-34s %6.2f %6.2f %6.2f %6.2f   %6.2f %6.2f %6.2f %6.2f   %.2f %.2f %.2f %.2f\n", r.name.c_str(),
               r.cyc[0], r.cyc[1], r.cyc[2], r.cyc[3], r.span[0], r.span[1], r.span[2], r.span[3], r.ghz[0], r.ghz[1],
               r.ghz[2], r.ghz[3]);
    if (json) {
        FILE* f = fopen(json, "w");
        if (!f) return 1;
        fprintf(f, "{\"device\": \"%s\", \"cus\": %d, \"method\": \"tools/ubench/rates.hip: 8 independent chains per "
                   "wave, grid = CUs x 4 SIMDs x W waves, median per-wave s_memtime cycles / (instructions x W)\", "
                   "\"waves_per_simd\": [1, 2, 4, 8], \"cycles_per_wave64_instr\": {",
                pr.gcnArchName, cus);
        for (size_t i = 0; i < rows.size(); ++i)
            fprintf(f, "%s\"%s\": [%.3f, %.3f, %.3f, %.3f]", i ? ", " : "", rows[i].name.c_str(), rows[i].cyc[0],
                    rows[i].cyc[1], rows[i].cyc[2], rows[i].cyc[3]);
        fprintf(f, "}, \"cycles_per_wave64_instr_span\": {");
        for (size_t i = 0; i < rows.size(); ++i)
            fprintf(f, "%s\"%s\": [%.3f, %.3f, %.3f, %.3f]", i ? ", " : "", rows[i].name.c_str(), rows[i].span[0],
                    rows[i].span[1], rows[i].span[2], rows[i].span[3]);
        fprintf(f, "}, \"ghz\": {");
        for (size_t i = 0; i < rows.size(); ++i)
            fprintf(f, "%s\"%s\": [%.3f, %.3f, %.3f, %.3f]", i ? ", " : "", rows[i].name.c_str(), rows[i].ghz[0],
                    rows[i].ghz[1], rows[i].ghz[2], rows[i].ghz[3]);
        fprintf(f, "}}\n");
        fclose(f);
    }
    return 0;
}
