// Fr-multiplier microbenchmark: throughput (many waves) and single-wave
// latency of candidate multipliers + correctness against lsp::fr_mul.
#include <cstdio>
#include <vector>
#include "mul_variants.hpp"
using namespace lsp;

template <int V> __device__ __forceinline__ Fr MUL(const Fr& a, const Fr& b) {
    if constexpr (V == 0) return fr_mul_cios(a, b);
    else if constexpr (V == 1) return fr_mul(a, b);
    else return lspx::mul_fips_asm(a, b);
}

template <int V> __global__ __launch_bounds__(256) void kthr(Fr* out, uint32_t iters) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    Fr a = fr_from_u64(t + 3), b = fr_from_u64(t * 7 + 5), c = fr_from_u64(t + 11), d = fr_from_u64(t + 13);
    const Fr m = fr_from_u64(0x1234567u + (uint32_t)t);
    for (uint32_t i = 0; i < iters; ++i) { a = MUL<V>(a, m); b = MUL<V>(b, m); c = MUL<V>(c, m); d = MUL<V>(d, m); }
    out[t] = fr_add(fr_add(a, b), fr_add(c, d));
}
template <int V> __global__ void klat(Fr* out, uint32_t iters) {
    Fr a = fr_from_u64(threadIdx.x + 3);
    const Fr m = fr_from_u64(0x1234567u + threadIdx.x);
    for (uint32_t i = 0; i < iters; ++i) a = MUL<V>(a, m);
    out[threadIdx.x] = a;
}
template <int V> __global__ void kcheck(const Fr* a, const Fr* b, Fr* out, size_t n) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t < n) out[t] = MUL<V>(a[t], b[t]);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int V> int run(const char* name, Fr* dout, Fr* da, Fr* db, Fr* dref, size_t n) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const size_t nth = 256 * 256 * 16; const uint32_t it = 256;
    hipLaunchKernelGGL(kthr<V>, dim3(nth / 256), dim3(256), 0, 0, dout, 4u);
    CK(hipDeviceSynchronize());
    hipEventRecord(e0); hipLaunchKernelGGL(kthr<V>, dim3(nth / 256), dim3(256), 0, 0, dout, it); hipEventRecord(e1);
    CK(hipEventSynchronize(e1)); float ms; hipEventElapsedTime(&ms, e0, e1);
    double gmul = (double)nth * it * 4 / (ms * 1e-3) / 1e9;
    const uint32_t lit = 4096;
    hipEventRecord(e0); hipLaunchKernelGGL(klat<V>, dim3(1), dim3(64), 0, 0, dout, lit); hipEventRecord(e1);
    CK(hipEventSynchronize(e1)); float lms; hipEventElapsedTime(&lms, e0, e1);
    hipLaunchKernelGGL(kcheck<V>, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, dout, n);
    CK(hipDeviceSynchronize());
    std::vector<Fr> got(n), ref(n);
    hipMemcpy(got.data(), dout, n * sizeof(Fr), hipMemcpyDeviceToHost);
    hipMemcpy(ref.data(), dref, n * sizeof(Fr), hipMemcpyDeviceToHost);
    size_t bad = 0; for (size_t i = 0; i < n; ++i) bad += !fr_eq(got[i], ref[i]);
    printf("%-12s throughput %7.1f G mul/s   single-wave latency %7.1f ns/mul   mismatches %zu/%zu\n", name, gmul,
           lms * 1e6 / lit, bad, n);
    return 0;
}

int main() {
    const size_t n = 1 << 20;
    std::vector<Fr> a(n), b(n);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    auto nx = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    for (size_t i = 0; i < n; ++i) {
        Fr x, y;
        for (int k = 0; k < 8; ++k) { x.v[k] = (uint32_t)nx(); y.v[k] = (uint32_t)nx(); }
        x.v[7] &= 0x0fffffffu; y.v[7] &= 0x0fffffffu;  // < r
        if (i < 16) { for (int k = 0; k < 8; ++k) { x.v[k] = mod_word(k); y.v[k] = mod_word(k); } x.v[0] -= 1 + (uint32_t)i; y.v[0] -= 1; }
        a[i] = x; b[i] = y;
    }
    Fr *da, *db, *dout, *dref;
    CK(hipMalloc(&da, n * sizeof(Fr))); CK(hipMalloc(&db, n * sizeof(Fr)));
    CK(hipMalloc(&dout, 256 * 256 * 16 * sizeof(Fr))); CK(hipMalloc(&dref, n * sizeof(Fr)));
    hipMemcpy(da, a.data(), n * sizeof(Fr), hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), n * sizeof(Fr), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kcheck<0>, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, dref, n);
    CK(hipDeviceSynchronize());
    // host check of the reference on a sample
    std::vector<Fr> ref(64); hipMemcpy(ref.data(), dref, 64 * sizeof(Fr), hipMemcpyDeviceToHost);
    size_t hb = 0; for (int i = 0; i < 64; ++i) hb += !fr_eq(ref[i], fr_mul(a[i], b[i]));
    printf("device vs host fr_mul mismatches: %zu/64\n", hb);
    run<0>("cios", dout, da, db, dref, n);
    run<1>("fips_col_asm", dout, da, db, dref, n);
    run<2>("fips_asm", dout, da, db, dref, n);
    return 0;
}
