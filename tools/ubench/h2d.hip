// Host -> device upload rates for the trace a drop-in `prove` receives in host
// memory (bin/src/main.rs:72,80-86: a host RowMajorMatrix).  One 2^19 x 8
// trace = 134 MB.  Modes (median of R runs, GB/s = bytes / wall time of the
// whole upload, synchronised):
//   pageable      hipMemcpyAsync from malloc'd memory (what lsp_prove did in round 4)
//   pinned        hipMemcpyAsync from hipHostMalloc'd memory (the DMA ceiling)
//   pinned2       the same split over two streams (two SDMA queues)
//   kernel        a copy kernel reading the pinned buffer over PCIe (zero-copy)
//   register      hipHostRegister + hipMemcpyAsync + hipHostUnregister per upload
//   register_fresh the same on a newly malloc'd and written buffer every run
//   ring:T:C:K    T host threads memcpy C-MiB chunks into K pinned slots while
//                 chunk k-1 is in flight (double-buffered staging)
// Usage: h2d [MiB] [runs]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

template <class F>
static double median_gbs(size_t bytes, int runs, F&& f) {
    std::vector<double> t;
    f();  // warm-up
    for (int r = 0; r < runs; ++r) {
        const double t0 = now();
        f();
        t.push_back(now() - t0);
    }
    std::sort(t.begin(), t.end());
    return bytes / t[t.size() / 2] / 1e9;
}

struct Ring {
    int T, K;
    size_t C;
    std::vector<void*> slot;
    std::vector<hipEvent_t> ev;  // one per chunk index (recorded after its DMA)
    hipStream_t st;
};

static void ring_upload(Ring& R, const char* src, char* dst, size_t bytes) {
    const size_t nch = (bytes + R.C - 1) / R.C;
    std::vector<std::atomic<int>> ready(nch), issued(nch);
    for (size_t j = 0; j < nch; ++j) ready[j] = 0, issued[j] = 0;
    if (R.ev.size() < nch) {
        size_t o = R.ev.size();
        R.ev.resize(nch);
        for (size_t j = o; j < nch; ++j) CK(hipEventCreateWithFlags(&R.ev[j], hipEventDisableTiming));
    }
    std::vector<std::thread> th;
    for (int t = 0; t < R.T; ++t)
        th.emplace_back([&, t] {
            for (size_t j = t; j < nch; j += R.T) {
                if (j >= (size_t)R.K) {  // the slot's previous chunk must have left
                    while (!issued[j - R.K].load(std::memory_order_acquire)) std::this_thread::yield();
                    CK(hipEventSynchronize(R.ev[j - R.K]));
                }
                const size_t n = std::min(R.C, bytes - j * R.C);
                std::memcpy(R.slot[j % R.K], src + j * R.C, n);
                ready[j].store(1, std::memory_order_release);
            }
        });
    for (size_t j = 0; j < nch; ++j) {
        while (!ready[j].load(std::memory_order_acquire)) std::this_thread::yield();
        const size_t n = std::min(R.C, bytes - j * R.C);
        CK(hipMemcpyAsync(dst + j * R.C, R.slot[j % R.K], n, hipMemcpyHostToDevice, R.st));
        CK(hipEventRecord(R.ev[j], R.st));
        issued[j].store(1, std::memory_order_release);
    }
    for (auto& x : th) x.join();
    CK(hipStreamSynchronize(R.st));
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 128;
    const int runs = argc > 2 ? std::atoi(argv[2]) : 9;
    const size_t bytes = mib << 20;
    char* pageable = (char*)std::malloc(bytes);
    for (size_t i = 0; i < bytes; ++i) pageable[i] = (char)(i * 131);
    char *pinned = nullptr, *dst = nullptr;
    CK(hipHostMalloc((void**)&pinned, bytes, hipHostMallocDefault));
    std::memcpy(pinned, pageable, bytes);
    CK(hipMalloc(&dst, bytes));
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    std::printf("{\"bytes\": %zu", bytes);
    std::printf(", \"pageable\": %.2f", median_gbs(bytes, runs, [&] {
                    CK(hipMemcpyAsync(dst, pageable, bytes, hipMemcpyHostToDevice, s0));
                    CK(hipStreamSynchronize(s0));
                }));
    std::printf(", \"pinned\": %.2f", median_gbs(bytes, runs, [&] {
                    CK(hipMemcpyAsync(dst, pinned, bytes, hipMemcpyHostToDevice, s0));
                    CK(hipStreamSynchronize(s0));
                }));
    std::printf(", \"pinned2\": %.2f", median_gbs(bytes, runs, [&] {
                    CK(hipMemcpyAsync(dst, pinned, bytes / 2, hipMemcpyHostToDevice, s0));
                    CK(hipMemcpyAsync(dst + bytes / 2, pinned + bytes / 2, bytes - bytes / 2, hipMemcpyHostToDevice, s1));
                    CK(hipStreamSynchronize(s0));
                    CK(hipStreamSynchronize(s1));
                }));
    {
        uint4* dp = nullptr;
        CK(hipHostGetDevicePointer((void**)&dp, pinned, 0));
        std::printf(", \"kernel\": %.2f", median_gbs(bytes, runs, [&] {
                        hipLaunchKernelGGL(k_copy, dim3(2048), dim3(256), 0, s0, dp, (uint4*)dst, bytes / 16);
                        CK(hipStreamSynchronize(s0));
                    }));
    }
    std::printf(", \"register\": %.2f", median_gbs(bytes, runs, [&] {
                    CK(hipHostRegister(pageable, bytes, hipHostRegisterDefault));
                    CK(hipMemcpyAsync(dst, pageable, bytes, hipMemcpyHostToDevice, s0));
                    CK(hipStreamSynchronize(s0));
                    CK(hipHostUnregister(pageable));
                }));
    {  // a fresh, written buffer each run: first-time page locking (a caller's new Vec)
        std::vector<double> t;
        for (int r = 0; r < runs; ++r) {
            char* f = (char*)std::malloc(bytes);
            std::memcpy(f, pageable, bytes);
            const double t0 = now();
            CK(hipHostRegister(f, bytes, hipHostRegisterDefault));
            const double t1 = now();
            CK(hipMemcpyAsync(dst, f, bytes, hipMemcpyHostToDevice, s0));
            CK(hipStreamSynchronize(s0));
            CK(hipHostUnregister(f));
            t.push_back(now() - t0);
            if (r == 0) std::printf(", \"register_fresh_only_ms\": %.3f", (t1 - t0) * 1e3);
            std::free(f);
        }
        std::sort(t.begin(), t.end());
        std::printf(", \"register_fresh\": %.2f", bytes / t[t.size() / 2] / 1e9);
    }
    {
        const double t0 = now();
        CK(hipHostRegister(pageable, bytes, hipHostRegisterDefault));
        const double t1 = now();
        CK(hipHostUnregister(pageable));
        std::printf(", \"register_only_ms\": %.3f, \"unregister_ms\": %.3f", (t1 - t0) * 1e3, (now() - t1) * 1e3);
    }
    std::printf(", \"host_memcpy_1t\": %.2f", median_gbs(bytes, runs, [&] { std::memcpy(pinned, pageable, bytes); }));
    const int Ts[] = {4, 8, 16};
    const size_t Cs[] = {4, 8, 16};
    for (int T : Ts)
        for (size_t C : Cs) {
            Ring R;
            R.T = T;
            R.K = 2 * T;
            R.C = C << 20;
            R.st = s0;
            for (int k = 0; k < R.K; ++k) {
                void* p = nullptr;
                CK(hipHostMalloc(&p, R.C, hipHostMallocDefault));
                R.slot.push_back(p);
            }
            std::printf(", \"ring:%d:%zu:%d\": %.2f", T, C, R.K,
                        median_gbs(bytes, runs, [&] { ring_upload(R, pageable, dst, bytes); }));
            for (void* p : R.slot) CK(hipHostFree(p));
            for (auto e : R.ev) CK(hipEventDestroy(e));
        }
    // device-side copy rate, for scale
    char* dst2 = nullptr;
    CK(hipMalloc(&dst2, bytes));
    std::printf(", \"d2d\": %.2f", median_gbs(2 * bytes, runs, [&] {
                    CK(hipMemcpyAsync(dst2, dst, bytes, hipMemcpyDeviceToDevice, s0));
                    CK(hipStreamSynchronize(s0));
                }));
    std::printf("}\n");
    std::fflush(stdout);
    CK(hipFree(dst2));
    CK(hipFree(dst));
    CK(hipHostFree(pinned));
    std::free(pageable);
    return 0;
}
