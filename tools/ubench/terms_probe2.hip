// Diagnostic: k_lookup_terms' body compiled standalone, with and without hipcub.
#include <hip/hip_runtime.h>
#ifdef WITH_HIPCUB
#include <hipcub/hipcub.hpp>
#endif
#include <cstdio>
#include <vector>
#include "fr.hpp"
using namespace lsp;
__device__ __forceinline__ bool fr_nonzero(const Fr& x) {
    uint32_t o = 0;
    for (int k = 0; k < 8; ++k) o |= x.v[k];
    return o != 0;
}
__global__ __launch_bounds__(256) void k_terms(const Fr* __restrict__ inv, const uint32_t* __restrict__ occ,
                                               const Fr* __restrict__ afil, size_t n, uint32_t nt,
                                               Fr* __restrict__ out, size_t ostride, uint32_t col_ainv,
                                               Fr* __restrict__ term) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr* row = out + i * ostride;
    const Fr ai = inv[i];
    row[col_ainv] = ai;
    Fr s = fr_nonzero(afil[i]) ? ai : fr_zero();
    for (uint32_t t = 0; t < nt; ++t) {
        const Fr bi = inv[(1 + (size_t)t) * n + i];
        const Fr o = fr_from_u64(occ[(size_t)t * n + i]);
        row[col_ainv + 1 + t] = bi;
        row[col_ainv + 1 + nt + t] = o;
        s = fr_sub(s, fr_mul(o, bi));
    }
    term[i] = s;
}
int main() {
    const size_t n = 8;
    std::vector<Fr> inv(2 * n, fr_one()), afil(n, fr_one()), out(n * 8, fr_zero());
    std::vector<uint32_t> occ = {4, 0, 0, 0, 0, 2, 0, 2};
    Fr *dinv, *dafil, *dout, *dterm; uint32_t* docc;
    hipMalloc(&dinv, inv.size() * 32); hipMalloc(&dafil, n * 32); hipMalloc(&dout, out.size() * 32);
    hipMalloc(&dterm, n * 32); hipMalloc(&docc, n * 4);
    hipMemcpy(dinv, inv.data(), inv.size() * 32, hipMemcpyHostToDevice);
    hipMemcpy(dafil, afil.data(), n * 32, hipMemcpyHostToDevice);
    hipMemcpy(docc, occ.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dout, out.data(), out.size() * 32, hipMemcpyHostToDevice);
    k_terms<<<1, 256>>>(dinv, docc, dafil, n, 1, dout, 8, 4, dterm);
    hipMemcpy(out.data(), dout, out.size() * 32, hipMemcpyDeviceToHost);
    int bad = 0;
    for (size_t i = 0; i < n; ++i) if (!fr_eq(out[i * 8 + 6], fr_from_u64(occ[i]))) ++bad;
    printf("terms probe: %d bad\n", bad);
}
