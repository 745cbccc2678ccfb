// Bounds-checked debug kernels ("device: bounds-checked debug
// kernels"; `python -m linea_stark_prover_amd.build --debug-bounds` defines
// LSP_DEBUG_BOUNDS and links liblsp_hip_dbg.so).
//
// LSP_BOUNDS(cond) is the constant `true` in the product build.  In the debug
// build a false condition records where it failed -- (file code << 16) | line,
// the first failure of a call wins -- in this translation unit's fault word and
// evaluates to false, so the caller skips the access instead of making it.  The
// kernel never faults (a faulting kernel can take every GPU of a node down) and
// never traps; the host reads every translation unit's word after each C-ABI
// call and fails that call with LSP_E_STATE "device bounds check failed at
// k_ntt.hip:123" (capi.cpp, bounds_fault_report).
//
// One fault word per translation unit for the whole process: the debug
// library is meant for one context (one stream) at a time.  With several
// contexts working at once (proofs in flight, the virtual ranks of an
// lsp_prove_group) a failed check in one context's kernel may be read, cleared
// and reported by another context's call, and the first call then returns
// LSP_OK; the debug suites (tests/test_gpu_debug_bounds.py, the parity suites
// under LSP_LIB=liblsp_hip_dbg.so) run one context at a time, and a group's
// failure is still reported by one of its ranks.
//
// The checks compare indices derived from launch geometry (tile position,
// row, column, LDS slot, table entry) with the extents the launch was planned
// for, and value-derived indices (the reduction table's quotient digit) with
// their table: what would otherwise read or write another buffer.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lsp {
namespace dbg {
// 15-bit code of a source file name (the host maps codes back to names)
constexpr uint32_t file_code(const char* s) {
    uint32_t h = 0;
    while (*s) h = h * 31u + (uint8_t)*s++;
    return h & 0x7fffu;
}
}  // namespace dbg
}  // namespace lsp

#ifdef LSP_DEBUG_BOUNDS
namespace lsp {
namespace dbg {
static __device__ unsigned int g_fault;  // one per translation unit
__device__ __noinline__ inline bool fail(unsigned where) {
    atomicCAS(&g_fault, 0u, where);  // a vector-memory atomic
    return false;
}
}  // namespace dbg
}  // namespace lsp
#define LSP_BOUNDS(cond) \
    ((cond) ? true : ::lsp::dbg::fail((::lsp::dbg::file_code(__FILE_NAME__) << 16) | (unsigned)__LINE__))
// the host reader of this translation unit's fault word (read and cleared)
#define LSP_BOUNDS_READER(NAME)                                                               \
    namespace lsp {                                                                           \
    unsigned bounds_fault_##NAME() {                                                          \
        unsigned v = 0, z = 0;                                                                \
        if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(dbg::g_fault), sizeof v) != hipSuccess) return 0; \
        if (v) (void)hipMemcpyToSymbol(HIP_SYMBOL(dbg::g_fault), &z, sizeof z);               \
        return v;                                                                             \
    }                                                                                         \
    }
#else
#define LSP_BOUNDS(cond) true
#define LSP_BOUNDS_READER(NAME)
#endif
