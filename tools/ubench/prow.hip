// The row-form compression (poseidon2_row.hpp) against the quad form the narrow
// Merkle levels run today (compress_f29<11, 4>), on one MI355X:
//   parity   digests of 4096 random pairs (and edge inputs 0, 1, r - 1) against
//            compress_f29<11, 1>, random round constants
//   latency  one wave alone, a chain of dependent compressions (s_memtime)
//   levels   a level of n = 512 .. 8192 nodes as the prover launches it:
//            quad form 16 nodes per 64-lane block, row form one node per wave
//   build: tools/ubench/build.sh prow    run: tools/ubench/prow
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <hip/hip_runtime.h>
#include "../../linea_stark_prover_amd/csrc/poseidon2_row.hpp"
using namespace lsp;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr uint32_t RF = 8, RP = 22;

__global__ void k_rc(const Fr* in, F29* rc29, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) rc29[i] = f29_from_fr(in[i]);
}

__global__ __launch_bounds__(256) void k_ref(const Fr* in, Fr* out, uint32_t n, const F29* rc29) {
    __shared__ uint4 qt[3 * F29_QTAB_N];
    f29_qtab_init(qt);
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = compress_f29<11, 1>(in[2 * i], in[2 * i + 1], rc29, RF, RP, qt);
}

__global__ __launch_bounds__(64) void k_row(const Fr* in, Fr* out, uint32_t n, const F29* rc29) {
    __shared__ prow::RowLds tab;
    prow::row_lds_init(&tab);
    __syncthreads();
    const uint32_t i = blockIdx.x;
    if (i >= n) return;
    const Fr d = prow::compress_row<11>(in + 2 * i, in + 2 * i + 1, rc29, RF, RP, &tab);
    if (threadIdx.x == 0) out[i] = d;
}

__global__ __launch_bounds__(64) void k_quad(const Fr* in, Fr* out, uint32_t n, const F29* rc29) {
    __shared__ uint4 qt[3 * F29_QTAB_N];
    f29_qtab_init(qt);
    __syncthreads();
    const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) / 4;
    if (i >= n) return;
    const Fr d = compress_f29<11, 4>(in[2 * i], in[2 * i + 1], rc29, RF, RP, qt);
    if ((threadIdx.x & 3) == 0) out[i] = d;
}

__global__ __launch_bounds__(64) void k_row_lat(const Fr* in, Fr* out, const F29* rc29, int iters, uint64_t* cyc) {
    __shared__ prow::RowLds tab;
    __shared__ Fr cur;
    prow::row_lds_init(&tab);
    if (threadIdx.x == 0) cur = in[0];
    __syncthreads();
    const uint64_t t0 = clock64();
    for (int k = 0; k < iters; ++k) {
        const Fr d = prow::compress_row<11>(&cur, in + 1, rc29, RF, RP, &tab);
        __syncthreads();
        if (threadIdx.x == 0) cur = d;
        __syncthreads();
    }
    const uint64_t t1 = clock64();
    if (threadIdx.x == 0) {
        out[0] = cur;
        cyc[0] = t1 - t0;
    }
}

__global__ __launch_bounds__(64) void k_quad_lat(const Fr* in, Fr* out, const F29* rc29, int iters, uint64_t* cyc) {
    __shared__ uint4 qt[3 * F29_QTAB_N];
    f29_qtab_init(qt);
    __syncthreads();
    Fr cur = in[0];
    const uint64_t t0 = clock64();
    for (int k = 0; k < iters; ++k) cur = compress_f29<11, 4>(cur, in[1], rc29, RF, RP, qt);
    const uint64_t t1 = clock64();
    if (threadIdx.x == 0) {
        out[0] = cur;
        cyc[0] = t1 - t0;
    }
}

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static uint32_t rnd() {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (uint32_t)(rng >> 11);
}
static Fr rand_fr() {  // < r: top word below r's (0x12ab655e)
    Fr x;
    for (int i = 0; i < 8; ++i) x.v[i] = rnd();
    x.v[7] &= 0x0fffffffu;
    return x;
}

int main() {
    const uint32_t nrc = 3 * RF + RP, N = 4096 + 3;
    std::vector<Fr> hrc(nrc), hin(2 * N);
    for (auto& x : hrc) x = rand_fr();
    for (auto& x : hin) x = rand_fr();
    // edge inputs: (0, 0), (1, r - 1), (r - 1, r - 1) in ark words
    const uint32_t rm1[8] = {0x00000000u, 0x0a118000u, 0xd0000001u, 0x59aa76feu,
                             0x5c37b001u, 0x60b44d1eu, 0x9a2ca556u, 0x12ab655eu};
    Fr Rm1, one{}, zero{};
    for (int i = 0; i < 8; ++i) Rm1.v[i] = rm1[i];
    one.v[0] = 1;
    hin[2 * 4096] = zero; hin[2 * 4096 + 1] = zero;
    hin[2 * 4097] = one; hin[2 * 4097 + 1] = Rm1;
    hin[2 * 4098] = Rm1; hin[2 * 4098 + 1] = Rm1;
    Fr *drc, *din, *dref, *drow, *dq, *dlat;
    F29* rc29;
    uint64_t* cyc;
    CK(hipMalloc(&drc, nrc * sizeof(Fr))); CK(hipMalloc(&rc29, nrc * sizeof(F29)));
    CK(hipMalloc(&din, 2 * N * sizeof(Fr))); CK(hipMalloc(&dref, N * sizeof(Fr)));
    CK(hipMalloc(&drow, N * sizeof(Fr))); CK(hipMalloc(&dq, N * sizeof(Fr)));
    CK(hipMalloc(&dlat, 4 * sizeof(Fr))); CK(hipMalloc(&cyc, 8));
    CK(hipMemcpy(drc, hrc.data(), nrc * sizeof(Fr), hipMemcpyHostToDevice));
    CK(hipMemcpy(din, hin.data(), 2 * N * sizeof(Fr), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_rc, dim3(1), dim3(64), 0, 0, drc, rc29, nrc);
    hipLaunchKernelGGL(k_ref, dim3((N + 255) / 256), dim3(256), 0, 0, din, dref, N, rc29);
    hipLaunchKernelGGL(k_row, dim3(N), dim3(64), 0, 0, din, drow, N, rc29);
    hipLaunchKernelGGL(k_quad, dim3((4 * N + 63) / 64), dim3(64), 0, 0, din, dq, N, rc29);
    CK(hipDeviceSynchronize());
    std::vector<Fr> a(N), b(N), c(N);
    CK(hipMemcpy(a.data(), dref, N * sizeof(Fr), hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), drow, N * sizeof(Fr), hipMemcpyDeviceToHost));
    CK(hipMemcpy(c.data(), dq, N * sizeof(Fr), hipMemcpyDeviceToHost));
    int bad_row = 0, bad_quad = 0;
    for (uint32_t i = 0; i < N; ++i) {
        bool er = false, eq = false;
        for (int w = 0; w < 8; ++w) {
            er |= a[i].v[w] != b[i].v[w];
            eq |= a[i].v[w] != c[i].v[w];
        }
        if (er && bad_row < 3) printf("row mismatch at %u: %08x.. vs %08x..\n", i, a[i].v[7], b[i].v[7]);
        bad_row += er;
        bad_quad += eq;
    }
    printf("parity over %u compressions (4096 random + edges): row form %d mismatches, quad form %d\n", N, bad_row,
           bad_quad);
    const int it = 20;
    for (int rep = 0; rep < 2; ++rep) {
        uint64_t cr, cq;
        hipLaunchKernelGGL(k_row_lat, dim3(1), dim3(64), 0, 0, din, dlat, rc29, it, cyc);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(&cr, cyc, 8, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL(k_quad_lat, dim3(1), dim3(64), 0, 0, din, dlat + 1, rc29, it, cyc);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(&cq, cyc, 8, hipMemcpyDeviceToHost));
        printf("one wave alone, clock64 ticks per dependent compression: quad form %.0f, row form %.0f (%.2fx)\n",
               (double)cq / it, (double)cr / it, (double)cq / cr);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (uint32_t n = 512; n <= 8192; n *= 2) {
        float tq = 1e9f, tr = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
            float ms;
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_quad, dim3((4 * n + 63) / 64), dim3(64), 0, 0, din, dq, n, rc29);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
            tq = ms < tq ? ms : tq;
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_row, dim3(n), dim3(64), 0, 0, din, drow, n, rc29);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
            tr = ms < tr ? ms : tr;
        }
        printf("level of %5u nodes: quad form %.1f us, row form %.1f us (%.2fx)\n", n, tq * 1e3, tr * 1e3, tq / tr);
    }
    return 0;
}
