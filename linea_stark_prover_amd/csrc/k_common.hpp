// Small device helpers shared by the kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "dbg_bounds.hpp"
#include "fr.hpp"

namespace lsp {

__device__ __forceinline__ uint64_t brev_bits(uint64_t x, uint32_t bits) {
    return bits == 0 ? 0 : (__brevll(x) >> (64 - bits));
}

// base^e from a two-level table {base^j, j < 2^L1} ++ {base^(j 2^L1) * scale, j < 2^L2}
__device__ __forceinline__ Fr pow2l(const Fr* __restrict__ tab, uint32_t L1, uint64_t e) {
    const uint64_t lo = e & ((1ull << L1) - 1);
    uint64_t hi = e >> L1;
    // the high half holds 2^L2 <= 2^L1 entries (two_level: L2 = bits - L1 <= L1)
    if (!LSP_BOUNDS(hi < (1ull << L1))) hi = 0;
    return fr_mul(tab[lo], tab[(1ull << L1) + hi]);
}

__device__ __forceinline__ size_t gtid() { return (size_t)blockIdx.x * blockDim.x + threadIdx.x; }

inline unsigned nblocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace lsp
