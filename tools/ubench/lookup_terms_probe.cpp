// Diagnostic: launch_lookup_terms on known inputs (occ = 4, 2), raw words out.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "kernels.hpp"
using namespace lsp;
int main() {
    const size_t n = 8;
    const uint32_t nt = 1;
    std::vector<Fr> inv(2 * n, fr_one()), afil(n, fr_one()), out(n * 8, fr_zero()), term(n);
    std::vector<uint32_t> occ = {4, 0, 0, 0, 0, 2, 0, 2};
    Fr *dinv, *dafil, *dout, *dterm;
    uint32_t* docc;
    hipMalloc(&dinv, inv.size() * 32); hipMalloc(&dafil, n * 32); hipMalloc(&dout, out.size() * 32);
    hipMalloc(&dterm, n * 32); hipMalloc(&docc, n * 4);
    hipMemcpy(dinv, inv.data(), inv.size() * 32, hipMemcpyHostToDevice);
    hipMemcpy(dafil, afil.data(), n * 32, hipMemcpyHostToDevice);
    hipMemcpy(docc, occ.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dout, out.data(), out.size() * 32, hipMemcpyHostToDevice);
    hipError_t e = launch_lookup_terms(dinv, docc, dafil, n, nt, dout, 8, 4, dterm, 0);
    hipDeviceSynchronize();
    hipMemcpy(out.data(), dout, out.size() * 32, hipMemcpyDeviceToHost);
    printf("launch %d\n", (int)e);
    for (size_t i = 0; i < n; ++i) {
        const Fr g = out[i * 8 + 6], x = fr_from_u64(occ[i]);
        printf("row %zu occ %u  got %08x %08x ... %08x  exp %08x %08x ... %08x  %s\n", i, occ[i], g.v[0], g.v[1],
               g.v[7], x.v[0], x.v[1], x.v[7], fr_eq(g, x) ? "OK" : "BAD");
    }
}
