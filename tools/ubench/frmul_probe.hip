// Diagnostic: device fr_mul / fr_from_u64 vs the host product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "fr.hpp"
using namespace lsp;
__global__ void k_from(const uint32_t* x, Fr* out, int n) {
    int i = threadIdx.x;
    if (i < n) out[i] = fr_from_u64(x[i]);
}
__global__ void k_mul(const Fr* a, const Fr* b, Fr* out, int n) {
    int i = threadIdx.x;
    if (i < n) out[i] = fr_mul(a[i], b[i]);
}
int main() {
    const int n = 64;
    std::vector<uint32_t> x(n);
    std::vector<Fr> a(n), b(n), o(n);
    uint64_t s = 12345;
    auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(s >> 32); };
    for (int i = 0; i < n; ++i) {
        x[i] = i < 16 ? i : rnd();
        Fr c;
        for (int k = 0; k < 8; ++k) c.v[k] = rnd();
        c.v[7] &= 0x0fffffff;
        a[i] = c;
        for (int k = 0; k < 8; ++k) c.v[k] = (i % 3 == 0 && k > 0) ? 0 : rnd();
        c.v[7] &= 0x0fffffff;
        b[i] = c;
    }
    uint32_t* dx; Fr *da, *db, *dout;
    hipMalloc(&dx, n * 4); hipMalloc(&da, n * 32); hipMalloc(&db, n * 32); hipMalloc(&dout, n * 32);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(da, a.data(), n * 32, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), n * 32, hipMemcpyHostToDevice);
    k_from<<<1, 64>>>(dx, dout, n);
    hipMemcpy(o.data(), dout, n * 32, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) if (!fr_eq(o[i], fr_from_u64(x[i]))) { if (bad < 4) printf("from_u64(%u) BAD\n", x[i]); ++bad; }
    printf("from_u64: %d bad of %d\n", bad, n);
    k_mul<<<1, 64>>>(da, db, dout, n);
    hipMemcpy(o.data(), dout, n * 32, hipMemcpyDeviceToHost);
    bad = 0;
    for (int i = 0; i < n; ++i) if (!fr_eq(o[i], fr_mul(a[i], b[i]))) ++bad;
    printf("mul: %d bad of %d\n", bad, n);
}
