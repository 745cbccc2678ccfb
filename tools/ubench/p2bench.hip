// Poseidon2 / F29 microbenchmark: correctness of the 29-bit-limb arithmetic
// against the 32-bit product, and permutation throughput of both forms.
#include <cstdio>
#include <vector>
#include "../../linea_stark_prover_amd/csrc/poseidon2.hpp"
#include "../../linea_stark_prover_amd/csrc/poseidon2_f29.hpp"
using namespace lsp;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void kmul_check(const Fr* a, const Fr* b, Fr* o1, Fr* o2, size_t n) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    o1[t] = fr_mul(a[t], b[t]);
    F29 x = f29_from_fr(a[t]), y = f29_from_fr(b[t]);
    // stress lazy bounds: add a few multiples before multiplying
    F29 xs = f29_add(f29_add(x, x), f29_add(x, x));   // 4x
    F29 p = f29_mul(xs, y);                             // 4xy
    F29 q = f29_mul(f29_add(p, f29_mul(x, y)), f29_from_fr(fr_one()));  // 5xy
    o2[t] = f29_to_fr(q);
}
__global__ void kmul_ref5(const Fr* o1, Fr* o3, size_t n) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    Fr x = o1[t];
    o3[t] = fr_add(fr_add(fr_add(x, x), fr_add(x, x)), x);
}
__global__ void kconv_rc(const Fr* rc, F29* rc29, int n) {
    int t = threadIdx.x;
    if (t < n) rc29[t] = f29_from_fr(rc[t]);
}
__global__ void kperm_check(Fr* st, Fr* st2, const Fr* rc, const F29* rc29, size_t n) {
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt table
    f29_qtab_init(qt);
    __syncthreads();
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    Fr a = st[3 * t], b = st[3 * t + 1], c = st[3 * t + 2];
    permute3<11>(a, b, c, rc, 8, 22);
    st[3 * t] = a; st[3 * t + 1] = b; st[3 * t + 2] = c;
    F29 x = f29_from_fr(st2[3 * t]), y = f29_from_fr(st2[3 * t + 1]), z = f29_from_fr(st2[3 * t + 2]);
    permute3_f29<11>(x, y, z, rc29, 8, 22, qt);
    st2[3 * t] = f29_to_fr(x); st2[3 * t + 1] = f29_to_fr(y); st2[3 * t + 2] = f29_to_fr(z);
}
template <int V> __global__ __launch_bounds__(256) void kperm_thr(Fr* out, const Fr* rc, const F29* rc29, int iters) {
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt table
    f29_qtab_init(qt);
    __syncthreads();
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    Fr a = fr_from_u64(t), b = fr_from_u64(t + 1), c = fr_zero();
    for (int i = 0; i < iters; ++i) {
        if (V == 0) { permute3<11>(a, b, c, rc, 8, 22); }
        else { a = compress_f29<11>(a, b, rc29, 8, 22, qt); }
    }
    out[t] = fr_add(fr_add(a, b), c);
}
__global__ __launch_bounds__(256) void kf29_thr(Fr* out, int iters) {
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    F29 a = f29_from_fr(fr_from_u64(t + 3)), b = f29_from_fr(fr_from_u64(t + 5)), c = f29_from_fr(fr_from_u64(t + 7)),
        d = f29_from_fr(fr_from_u64(t + 9));
    const F29 m = f29_from_fr(fr_from_u64(0x1234567 + t));
    for (int i = 0; i < iters; ++i) { a = f29_mul(a, m); b = f29_mul(b, m); c = f29_mul(c, m); d = f29_mul(d, m); }
    out[t] = fr_add(fr_add(f29_to_fr(a), f29_to_fr(b)), fr_add(f29_to_fr(c), f29_to_fr(d)));
}
__global__ void kf29_lat(Fr* out, int iters) {
    F29 a = f29_from_fr(fr_from_u64(threadIdx.x + 3));
    const F29 m = f29_from_fr(fr_from_u64(0x1234567 + threadIdx.x));
    for (int i = 0; i < iters; ++i) a = f29_mul(a, m);
    out[threadIdx.x] = f29_to_fr(a);
}
template <int V> __global__ void kperm_lat(Fr* out, const Fr* rc, const F29* rc29, int iters) {
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt table
    f29_qtab_init(qt);
    __syncthreads();
    Fr a = fr_from_u64(threadIdx.x), b = fr_from_u64(threadIdx.x + 1), c = fr_zero();
    for (int i = 0; i < iters; ++i) {
        if (V == 0) permute3<11>(a, b, c, rc, 8, 22); else a = compress_f29<11>(a, b, rc29, 8, 22, qt);
    }
    out[threadIdx.x] = fr_add(fr_add(a, b), c);
}

__global__ void kcoop_lat(Fr* out, const F29* rc29, int iters) {
    __shared__ uint4 qt[3 * F29_QTAB_N];  // f29_reduce_qt table
    f29_qtab_init(qt);
    __syncthreads();
    Fr a = fr_from_u64(threadIdx.x >> 2), b = fr_from_u64((threadIdx.x >> 2) + 1);
    for (int i = 0; i < iters; ++i) a = compress_f29<11, true>(a, b, rc29, 8, 22, qt);
    out[threadIdx.x] = a;
}

static float timeit(void (*f)(void*), void* arg) { return 0; }

int main() {
    const size_t n = 1 << 20;
    std::vector<Fr> a(n), b(n);
    uint64_t s = 0x12345678abcdefull;
    auto nx = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    for (size_t i = 0; i < n; ++i) {
        for (int k = 0; k < 8; ++k) { a[i].v[k] = (uint32_t)nx(); b[i].v[k] = (uint32_t)nx(); }
        a[i].v[7] &= 0x0fffffffu; b[i].v[7] &= 0x0fffffffu;
        if (i < 8) { for (int k = 0; k < 8; ++k) a[i].v[k] = mod_word(k); a[i].v[0] -= 1 + (uint32_t)i; }
    }
    Fr *da, *db, *o1, *o2, *o3, *dst, *dst2, *drc, *dout; F29* drc29;
    CK(hipMalloc(&da, n * 32)); CK(hipMalloc(&db, n * 32)); CK(hipMalloc(&o1, n * 32)); CK(hipMalloc(&o2, n * 32));
    CK(hipMalloc(&o3, n * 32)); CK(hipMalloc(&dst, 3 * n * 32)); CK(hipMalloc(&dst2, 3 * n * 32));
    CK(hipMalloc(&drc, 46 * 32)); CK(hipMalloc(&drc29, 46 * sizeof(F29))); CK(hipMalloc(&dout, 256 * 256 * 16 * 32));
    CK(hipMemcpy(da, a.data(), n * 32, hipMemcpyHostToDevice)); CK(hipMemcpy(db, b.data(), n * 32, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(kmul_check, dim3(n / 256), dim3(256), 0, 0, da, db, o1, o2, n);
    hipLaunchKernelGGL(kmul_ref5, dim3(n / 256), dim3(256), 0, 0, o1, o3, n);
    CK(hipDeviceSynchronize());
    std::vector<Fr> r2(n), r3(n);
    CK(hipMemcpy(r2.data(), o2, n * 32, hipMemcpyDeviceToHost)); CK(hipMemcpy(r3.data(), o3, n * 32, hipMemcpyDeviceToHost));
    size_t bad = 0; for (size_t i = 0; i < n; ++i) bad += !fr_eq(r2[i], r3[i]);
    printf("f29 lazy mul/add chain vs 32-bit: mismatches %zu / %zu\n", bad, n);
    // permutation equality
    std::vector<Fr> rc(46); for (auto& x : rc) { for (int k = 0; k < 8; ++k) x.v[k] = (uint32_t)nx(); x.v[7] &= 0x0fffffffu; }
    CK(hipMemcpy(drc, rc.data(), 46 * 32, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(kconv_rc, dim3(1), dim3(64), 0, 0, drc, drc29, 46);
    std::vector<Fr> st(3 * n); for (size_t i = 0; i < 3 * n; ++i) st[i] = i % 3 == 0 ? a[i / 3] : (i % 3 == 1 ? b[i / 3] : a[(i / 3 + 7) % n]);
    CK(hipMemcpy(dst, st.data(), 3 * n * 32, hipMemcpyHostToDevice)); CK(hipMemcpy(dst2, st.data(), 3 * n * 32, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(kperm_check, dim3(n / 256), dim3(256), 0, 0, dst, dst2, drc, drc29, n);
    CK(hipDeviceSynchronize());
    std::vector<Fr> p1(3 * n), p2(3 * n);
    CK(hipMemcpy(p1.data(), dst, 3 * n * 32, hipMemcpyDeviceToHost)); CK(hipMemcpy(p2.data(), dst2, 3 * n * 32, hipMemcpyDeviceToHost));
    bad = 0; for (size_t i = 0; i < 3 * n; ++i) bad += !fr_eq(p1[i], p2[i]);
    printf("poseidon2 f29 vs 32-bit: mismatches %zu / %zu\n", bad, 3 * n);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); float ms;
    const size_t nth = 256 * 256 * 16;
    hipLaunchKernelGGL(kf29_thr, dim3(nth / 256), dim3(256), 0, 0, dout, 4); CK(hipDeviceSynchronize());
    (void)hipEventRecord(e0); hipLaunchKernelGGL(kf29_thr, dim3(nth / 256), dim3(256), 0, 0, dout, 256); (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("f29_mul throughput %.1f G mul/s\n", nth * 256.0 * 4 / (ms * 1e-3) / 1e9);
    (void)hipEventRecord(e0); hipLaunchKernelGGL(kf29_lat, dim3(1), dim3(64), 0, 0, dout, 4096); (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    printf("f29_mul single-wave latency %.1f ns/mul\n", ms * 1e6 / 4096);
    for (int v = 0; v < 2; ++v) {
        const size_t pt = 256 * 256 * 8; const int it = 8;
        if (v == 0) hipLaunchKernelGGL(kperm_thr<0>, dim3(pt / 256), dim3(256), 0, 0, dout, drc, drc29, 1);
        else hipLaunchKernelGGL(kperm_thr<1>, dim3(pt / 256), dim3(256), 0, 0, dout, drc, drc29, 1);
        CK(hipDeviceSynchronize());
        (void)hipEventRecord(e0);
        if (v == 0) hipLaunchKernelGGL(kperm_thr<0>, dim3(pt / 256), dim3(256), 0, 0, dout, drc, drc29, it);
        else hipLaunchKernelGGL(kperm_thr<1>, dim3(pt / 256), dim3(256), 0, 0, dout, drc, drc29, it);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
        double mps = pt * (double)it / (ms * 1e-3) / 1e6;
        (void)hipEventRecord(e0);
        if (v == 0) hipLaunchKernelGGL(kperm_lat<0>, dim3(1), dim3(64), 0, 0, dout, drc, drc29, 64);
        else hipLaunchKernelGGL(kperm_lat<1>, dim3(1), dim3(64), 0, 0, dout, drc, drc29, 64);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); float lms; (void)hipEventElapsedTime(&lms, e0, e1);
        printf("%s poseidon2: %.1f M perm/s (x230 = %.1f G mul/s)   single-wave latency %.1f us/perm\n",
               v == 0 ? "32-bit" : "f29   ", mps, mps * 230 / 1e3, lms * 1e3 / 64);
    }
    {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(kcoop_lat, dim3(1), dim3(64), 0, 0, dout, drc29, 64);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); float lms; (void)hipEventElapsedTime(&lms, e0, e1);
        printf("f29 quad-coop poseidon2 single-wave latency %.1f us/perm\n", lms * 1e3 / 64);
    }
    return 0;
}
