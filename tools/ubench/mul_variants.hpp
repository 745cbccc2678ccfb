// Candidate Montgomery multipliers for Fr (8 x 32-bit limbs), compared by
// tools/ubench/mulbench.hip.  All return canonical results.
#pragma once
#include "../../linea_stark_prover_amd/csrc/fr.hpp"

namespace lspx {
using lsp::Fr;
using lsp::mod_word;

// FIPS product scanning, C formulation: 3-word accumulator (acc64, acc2)
__device__ __forceinline__ Fr mul_fips_c(const Fr& a, const Fr& b) {
    uint32_t m[8], r[8];
    uint64_t acc = 0;
    uint32_t acc2 = 0;
#define MAC(x, y)                                                   \
    do {                                                            \
        uint64_t p_ = (uint64_t)(x) * (y);                          \
        uint64_t s_;                                                \
        acc2 += __builtin_add_overflow(acc, p_, &s_) ? 1u : 0u;     \
        acc = s_;                                                   \
    } while (0)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
        for (int j = 0; j < k; ++j) {
            MAC(a.v[j], b.v[k - j]);
            MAC(m[j], mod_word(k - j));
        }
        MAC(a.v[k], b.v[0]);
        m[k] = 0u - (uint32_t)acc;
        {
            uint64_t s_;
            acc2 += __builtin_add_overflow(acc, (uint64_t)m[k], &s_) ? 1u : 0u;
            acc = s_;
        }
        acc = (acc >> 32) | ((uint64_t)acc2 << 32);
        acc2 = 0;
    }
#pragma unroll
    for (int k = 8; k < 15; ++k) {
#pragma unroll
        for (int j = k - 7; j < 8; ++j) {
            MAC(a.v[j], b.v[k - j]);
            MAC(m[j], mod_word(k - j));
        }
        r[k - 8] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)acc2 << 32);
        acc2 = 0;
    }
    r[7] = (uint32_t)acc;
#undef MAC
    Fr o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o.v[i] = r[i];
    return lsp::fr_reduce_once(o);
}

// FIPS with inline asm: v_mad_u64_u32 with carry-out into an SGPR pair,
// v_addc_co_u32 to fold the carry into the third accumulator word.
__device__ __forceinline__ void mac_asm(uint64_t& acc, uint32_t& acc2, uint32_t x, uint32_t y) {
    uint64_t c;
    asm volatile(
        "v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
        "v_addc_co_u32_e64 %2, %1, %2, 0, %1"
        : "+v"(acc), "=&s"(c), "+v"(acc2)
        : "v"(x), "v"(y));
}
__device__ __forceinline__ void mac_asm_s(uint64_t& acc, uint32_t& acc2, uint32_t x, uint32_t ys) {
    uint64_t c;
    asm volatile(
        "v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
        "v_addc_co_u32_e64 %2, %1, %2, 0, %1"
        : "+v"(acc), "=&s"(c), "+v"(acc2)
        : "v"(x), "s"(ys));
}

__device__ __forceinline__ Fr mul_fips_asm(const Fr& a, const Fr& b) {
    uint32_t m[8], r[8];
    uint64_t acc = 0;
    uint32_t acc2 = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
        for (int j = 0; j < k; ++j) {
            mac_asm(acc, acc2, a.v[j], b.v[k - j]);
            mac_asm_s(acc, acc2, m[j], mod_word(k - j));
        }
        mac_asm(acc, acc2, a.v[k], b.v[0]);
        m[k] = 0u - (uint32_t)acc;
        // + m[k] * r[0] (= m[k]): low word becomes 0, carry = (low != 0)
        const uint32_t carry = (uint32_t)acc != 0u;
        acc = (acc >> 32) + carry + ((uint64_t)acc2 << 32);
        acc2 = 0;
    }
#pragma unroll
    for (int k = 8; k < 15; ++k) {
#pragma unroll
        for (int j = k - 7; j < 8; ++j) {
            mac_asm(acc, acc2, a.v[j], b.v[k - j]);
            mac_asm_s(acc, acc2, m[j], mod_word(k - j));
        }
        r[k - 8] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)acc2 << 32);
        acc2 = 0;
    }
    r[7] = (uint32_t)acc;
    Fr o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o.v[i] = r[i];
    return lsp::fr_reduce_once(o);
}
}  // namespace lspx
