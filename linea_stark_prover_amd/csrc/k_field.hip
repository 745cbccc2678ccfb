// Batch inversion (p3-field batch_multiplicative_inverse) and the gather used
// to pull query openings off the device in one copy.
#include "k_common.hpp"
#include "kernels.hpp"

namespace lsp {

namespace {
// Thread t owns elements t, t+T, t+2T, ... (`chunk` of them, interleaved so every
// pass is coalesced): a prefix product, one Fermat inverse, the back pass.  The
// inverse (~380 products) is one instruction stream per wave whatever the
// chunk, so the launcher sizes the chunk for about one wave per SIMD.
__global__ __launch_bounds__(256) void k_batch_inverse(const Fr* __restrict__ in, Fr* __restrict__ out, size_t n,
                                                       size_t T, uint32_t chunk) {
    const size_t t = gtid();
    if (t >= T) return;
    Fr acc = fr_one();
    uint32_t cnt = 0;
    for (uint32_t j = 0; j < chunk; ++j) {
        const size_t i = t + (size_t)j * T;
        if (i >= n) break;
        out[i] = acc;
        acc = fr_mul(acc, in[i]);
        ++cnt;
    }
    Fr inv = fr_inv(acc);
    for (uint32_t j = cnt; j-- > 0;) {
        const size_t i = t + (size_t)j * T;
        const Fr o = fr_mul(inv, out[i]);
        inv = fr_mul(inv, in[i]);
        out[i] = o;
    }
}

// Fr-mul throughput probe of the multiplier the Poseidon2 kernels use (the
// 29-bit-limb product, fr29.hpp): 4 independent register-resident chains per lane
__global__ __launch_bounds__(256) void k_calib_mul(Fr* __restrict__ out, uint32_t iters) {
    const size_t t = gtid();
    F29 a = f29_from_fr(fr_from_u64(t + 3)), b = f29_from_fr(fr_from_u64(t * 7 + 5)),
        c = f29_from_fr(fr_from_u64(t + 11)), d = f29_from_fr(fr_from_u64(t + 13));
    const F29 m = f29_from_fr(fr_from_u64(0x1234567u + (uint32_t)t));
    for (uint32_t i = 0; i < iters; ++i) {
        a = f29_mul(a, m);
        b = f29_mul(b, m);
        c = f29_mul(c, m);
        d = f29_mul(d, m);
    }
    out[t] = fr_add(fr_add(f29_to_fr(a), f29_to_fr(b)), fr_add(f29_to_fr(c), f29_to_fr(d)));
}

__global__ __launch_bounds__(256) void k_gather(const uint64_t* __restrict__ ptrs, Fr* __restrict__ out, size_t n) {
    const size_t i = gtid();
    if (i < n) out[i] = *reinterpret_cast<const Fr*>(ptrs[i]);
}

__global__ __launch_bounds__(256) void k_assemble_chunks(const Fr* __restrict__ stage, uint32_t logGq, size_t cpr,
                                                         size_t h, Fr* __restrict__ out) {
    const size_t t = gtid();
    const size_t q = cpr << logGq;
    if (t >= h * q) return;
    const size_t k = t / q, j = t - k * q;
    const size_t r = brev_bits(j & ((1ull << logGq) - 1), logGq), c = j >> logGq;
    out[t] = stage[(r * h + k) * cpr + c];
}
}  // namespace

hipError_t launch_batch_inverse(const Fr* in, Fr* out, size_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    // lanes for one wave per SIMD (256 CUs x 4 SIMDs x 64), 8 .. 256 elements each
    uint32_t chunk = 8;
    while (chunk < 256 && (size_t)chunk * 65536 < n) chunk *= 2;
    const size_t T = (n + chunk - 1) / chunk;
    hipLaunchKernelGGL(k_batch_inverse, dim3(nblocks(T, 256)), dim3(256), 0, st, in, out, n, T, chunk);
    return hipGetLastError();
}

hipError_t launch_calib_mul(Fr* out, size_t nthreads, uint32_t iters, hipStream_t st) {
    hipLaunchKernelGGL(k_calib_mul, dim3(nblocks(nthreads, 256)), dim3(256), 0, st, out, iters);
    return hipGetLastError();
}

hipError_t launch_gather(const uint64_t* ptrs, Fr* out, size_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gather, dim3(nblocks(n, 256)), dim3(256), 0, st, ptrs, out, n);
    return hipGetLastError();
}

hipError_t launch_assemble_chunks(const Fr* stage, uint32_t logGq, size_t cpr, size_t h, Fr* out, hipStream_t st) {
    const size_t n = h * (cpr << logGq);
    hipLaunchKernelGGL(k_assemble_chunks, dim3(nblocks(n, 256)), dim3(256), 0, st, stage, logGq, cpr, h, out);
    return hipGetLastError();
}

}  // namespace lsp
