// Poseidon2Bls12337<3> on the host, 8 permutations at a time with AVX-512 IFMA
// (vpmadd52luq / vpmadd52huq): the Merkle tree tops the host finishes
// (prove.cpp commit_device) are many independent compressions per level, so
// eight lanes of 52-bit multiply-adds cover eight of them for about the cost
// of one scalar 4 x 64-bit permutation (poseidon2_host64.hpp).
//
// Representation: 5 limbs of 52 bits per lane, Montgomery form with
// R = 2^260 (X = x 2^260 mod r).  Values stay lazily reduced in [0, 2r) exactly
// as in poseidon2_host64.hpp: a product of inputs < 2r is < 1.02 r (word-by-word
// Montgomery with 52-bit digits, no final subtraction; 4 r^2 / 2^260 < 0.02 r),
// a sum is reduced by one conditional subtraction of 2r.  Entry: the ark-form
// integer A = x 2^256 times 2^264 (Montgomery) = x 2^260; exit: X times 2^256 =
// x 2^256, made canonical.  Same permutation (U1-U3 conventions) as
// poseidon2.hpp; tests/test_host.py checks it against the oracle.
//
// Compiled for every x86-64 host; the IFMA functions carry their own target
// attribute and run only when the CPU reports avx512f + avx512ifma (EPYC Zen 4/5,
// recent Xeons), else the callers use the scalar path.
#include "host.hpp"

// host code only: the .cpp sources also go through hipcc's device pass
#ifndef __HIP_DEVICE_COMPILE__
#include <immintrin.h>

#include <cstdlib>
#include <cstring>

namespace lsp {
namespace ifma {
namespace {

#define LSP_IFMA __attribute__((target("avx512f,avx512ifma"), always_inline)) inline

constexpr uint64_t M52 = (1ull << 52) - 1;
constexpr uint64_t RL[5] = {0x1800000000001ull, 0xfed00000010a1ull, 0xc37b00159aa76ull, 0xa55660b44d1e5ull,
                            0x12ab655e9a2cull};
constexpr uint64_t R2L[5] = {0x3000000000002ull, 0xfda0000002142ull, 0x86f6002b354edull, 0x4aacc1689a3cbull,
                             0x2556cabd3459ull};
constexpr uint64_t NP52 = 0x17fffffffffffull;  // -r^-1 mod 2^52
constexpr uint64_t C264[5] = {0xefffffffff24aull, 0x481ffff1bff40ull, 0xc78cd7c98c476ull, 0x11ae17e6a1bb9ull,
                              0x60020ea1fddull};  // 2^264 mod r
constexpr uint64_t C256[5] = {0xc7ffffffffff3ull, 0xf6ffffff27d1ull, 0x12c0fee7257f5ull, 0x9a9d16d815755ull,
                              0xd4bda322bbbull};  // 2^256 mod r

struct V {
    __m512i l[5];
};

LSP_IFMA __m512i bc(uint64_t x) { return _mm512_set1_epi64((long long)x); }

LSP_IFMA V vconst(const uint64_t c[5]) {
    V v;
    for (int k = 0; k < 5; ++k) v.l[k] = bc(c[k]);
    return v;
}

// a b 2^-260 mod r, lazily (< 1.02 r for inputs < 2r); inputs with normalised limbs
LSP_IFMA V mul(const V& a, const V& b) {
    const __m512i z = _mm512_setzero_si512();
    const __m512i np = bc(NP52);
    const __m512i r0 = bc(RL[0]), r1 = bc(RL[1]), r2 = bc(RL[2]), r3 = bc(RL[3]), r4 = bc(RL[4]);
    __m512i t0 = z, t1 = z, t2 = z, t3 = z, t4 = z, t5 = z;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const __m512i bi = b.l[i];
        t0 = _mm512_madd52lo_epu64(t0, a.l[0], bi);
        t1 = _mm512_madd52lo_epu64(t1, a.l[1], bi);
        t2 = _mm512_madd52lo_epu64(t2, a.l[2], bi);
        t3 = _mm512_madd52lo_epu64(t3, a.l[3], bi);
        t4 = _mm512_madd52lo_epu64(t4, a.l[4], bi);
        t1 = _mm512_madd52hi_epu64(t1, a.l[0], bi);
        t2 = _mm512_madd52hi_epu64(t2, a.l[1], bi);
        t3 = _mm512_madd52hi_epu64(t3, a.l[2], bi);
        t4 = _mm512_madd52hi_epu64(t4, a.l[3], bi);
        t5 = _mm512_madd52hi_epu64(t5, a.l[4], bi);
        const __m512i m = _mm512_madd52lo_epu64(z, t0, np);
        t0 = _mm512_madd52lo_epu64(t0, m, r0);
        t1 = _mm512_madd52lo_epu64(t1, m, r1);
        t2 = _mm512_madd52lo_epu64(t2, m, r2);
        t3 = _mm512_madd52lo_epu64(t3, m, r3);
        t4 = _mm512_madd52lo_epu64(t4, m, r4);
        t1 = _mm512_madd52hi_epu64(t1, m, r0);
        t2 = _mm512_madd52hi_epu64(t2, m, r1);
        t3 = _mm512_madd52hi_epu64(t3, m, r2);
        t4 = _mm512_madd52hi_epu64(t4, m, r3);
        t5 = _mm512_madd52hi_epu64(t5, m, r4);
        // t0 = 0 mod 2^52 now: drop the digit
        t0 = _mm512_add_epi64(t1, _mm512_srli_epi64(t0, 52));
        t1 = t2;
        t2 = t3;
        t3 = t4;
        t4 = t5;
        t5 = z;
    }
    const __m512i mk = bc(M52);
    V o;
    t1 = _mm512_add_epi64(t1, _mm512_srli_epi64(t0, 52));
    o.l[0] = _mm512_and_si512(t0, mk);
    t2 = _mm512_add_epi64(t2, _mm512_srli_epi64(t1, 52));
    o.l[1] = _mm512_and_si512(t1, mk);
    t3 = _mm512_add_epi64(t3, _mm512_srli_epi64(t2, 52));
    o.l[2] = _mm512_and_si512(t2, mk);
    t4 = _mm512_add_epi64(t4, _mm512_srli_epi64(t3, 52));
    o.l[3] = _mm512_and_si512(t3, mk);
    o.l[4] = t4;
    return o;
}

// v - m if v >= m, else v (normalised limbs, m a constant)
LSP_IFMA V csub(const V& v, const uint64_t m[5]) {
    const __m512i mk = bc(M52);
    V d;
    __m512i c = _mm512_setzero_si512();
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const __m512i x = _mm512_add_epi64(_mm512_sub_epi64(v.l[k], bc(m[k])), c);
        if (k < 4) {
            c = _mm512_srai_epi64(x, 52);  // borrow: -1 or 0
            d.l[k] = _mm512_and_si512(x, mk);
        } else {
            d.l[k] = x;
        }
    }
    const __mmask8 neg = _mm512_cmplt_epi64_mask(d.l[4], _mm512_setzero_si512());
    V o;
#pragma unroll
    for (int k = 0; k < 5; ++k) o.l[k] = _mm512_mask_blend_epi64(neg, d.l[k], v.l[k]);
    return o;
}

// (a + b) for inputs < 2r, reduced below 2r
LSP_IFMA V add(const V& a, const V& b) {
    const __m512i mk = bc(M52);
    V s;
    __m512i c = _mm512_setzero_si512();
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const __m512i x = _mm512_add_epi64(_mm512_add_epi64(a.l[k], b.l[k]), c);
        if (k < 4) {
            c = _mm512_srli_epi64(x, 52);
            s.l[k] = _mm512_and_si512(x, mk);
        } else {
            s.l[k] = x;
        }
    }
    return csub(s, R2L);
}

// ark-form words (8 lanes; lane j at src[j * stride]) -> IFMA form
LSP_IFMA V load(const Fr* src, size_t stride, int n) {
    alignas(64) uint64_t t[5][8];
    for (int j = 0; j < 8; ++j) {
        uint64_t w[4] = {0, 0, 0, 0};
        if (j < n) std::memcpy(w, src + j * stride, 32);
        t[0][j] = w[0] & M52;
        t[1][j] = ((w[0] >> 52) | (w[1] << 12)) & M52;
        t[2][j] = ((w[1] >> 40) | (w[2] << 24)) & M52;
        t[3][j] = ((w[2] >> 28) | (w[3] << 36)) & M52;
        t[4][j] = w[3] >> 16;
    }
    V a;
    for (int k = 0; k < 5; ++k) a.l[k] = _mm512_load_si512(t[k]);
    return mul(a, vconst(C264));  // x 2^256 * 2^264 * 2^-260 = x 2^260
}

// IFMA form -> canonical ark-form words
LSP_IFMA void store(const V& x, Fr* dst, size_t stride, int n) {
    const V y = csub(mul(x, vconst(C256)), RL);  // x 2^256, < r
    alignas(64) uint64_t t[5][8];
    for (int k = 0; k < 5; ++k) _mm512_store_si512(t[k], y.l[k]);
    for (int j = 0; j < n; ++j) {
        uint64_t w[4];
        w[0] = t[0][j] | (t[1][j] << 52);
        w[1] = (t[1][j] >> 12) | (t[2][j] << 40);
        w[2] = (t[2][j] >> 24) | (t[3][j] << 28);
        w[3] = (t[3][j] >> 36) | (t[4][j] << 16);
        std::memcpy(dst + j * stride, w, 32);
    }
}

// two independent 8-lane states in lockstep: the dependent IFMA chains of one
// product leave the multiply pipes partly idle, the other state's fill them
struct W {
    V x, y;
};
LSP_IFMA W mul(const W& a, const W& b) { return W{mul(a.x, b.x), mul(a.y, b.y)}; }
LSP_IFMA W add(const W& a, const W& b) { return W{add(a.x, b.x), add(a.y, b.y)}; }
LSP_IFMA W add(const W& a, const V& c) { return W{add(a.x, c), add(a.y, c)}; }
LSP_IFMA W mul(const V& c, const W& a) { return W{mul(c, a.x), mul(c, a.y)}; }

template <uint32_t D, class T>
LSP_IFMA T sbox_t(const T& x) {
    const T x2 = mul(x, x);
#ifndef LSP_HOST_SBOX5  // x^3 and x^4 side by side: 4 dependent products (poseidon2_host64.hpp)
    if (D == 11) {
        const T x3 = mul(x2, x);
        const T x4 = mul(x2, x2);
        return mul(mul(x4, x4), x3);
    }
#endif
    const T x4 = mul(x2, x2);
    const T x8 = mul(x4, x4);
    if (D == 11) return mul(mul(x8, x2), x);
    return mul(mul(x8, x8), x);  // x^17
}

template <class T>
LSP_IFMA void ext_layer_t(T& s0, T& s1, T& s2) {
    const T t = add(add(s0, s1), s2);
    s0 = add(s0, t);
    s1 = add(s1, t);
    s2 = add(s2, t);
}

// caller-set U2/U3 layers (P2Layout::gen_lin; poseidon2_host64.hpp):
// m = M_E row-major [9], d = the internal diagonal [3], broadcast in V
template <class T>
LSP_IFMA void ext_layer_gen_t(T& s0, T& s1, T& s2, const V* m) {
    const T n0 = add(add(mul(m[0], s0), mul(m[1], s1)), mul(m[2], s2));
    const T n1 = add(add(mul(m[3], s0), mul(m[4], s1)), mul(m[5], s2));
    const T n2 = add(add(mul(m[6], s0), mul(m[7], s1)), mul(m[8], s2));
    s0 = n0;
    s1 = n1;
    s2 = n2;
}

// T = V (8 states) or W (16 states); round constants broadcast in V; lin:
// nullptr = the default U2/U3 layers, else M_E [9] then d [3]
template <uint32_t D, class T>
LSP_IFMA void permute(T& s0, T& s1, T& s2, const V* rc, uint32_t rounds_f, uint32_t rounds_p,
                      const V* lin = nullptr) {
    const uint32_t half = rounds_f / 2;
    const V* ini = rc;
    const V* ter = rc + 3 * half;
    const V* itl = rc + 6 * half;
    if (lin)
        ext_layer_gen_t(s0, s1, s2, lin);
    else
        ext_layer_t(s0, s1, s2);
    for (uint32_t r = 0; r < half; ++r) {
        s0 = sbox_t<D>(add(s0, ini[3 * r + 0]));
        s1 = sbox_t<D>(add(s1, ini[3 * r + 1]));
        s2 = sbox_t<D>(add(s2, ini[3 * r + 2]));
        if (lin)
            ext_layer_gen_t(s0, s1, s2, lin);
        else
            ext_layer_t(s0, s1, s2);
    }
    for (uint32_t r = 0; r < rounds_p; ++r) {
        s0 = sbox_t<D>(add(s0, itl[r]));
        const T t = add(add(s0, s1), s2);
        if (lin) {
            s0 = add(t, mul(lin[9], s0));
            s1 = add(t, mul(lin[10], s1));
            s2 = add(t, mul(lin[11], s2));
            continue;
        }
        s0 = add(s0, t);
        s1 = add(s1, t);
        s2 = add(add(s2, s2), t);
    }
    for (uint32_t r = 0; r < half; ++r) {
        s0 = sbox_t<D>(add(s0, ter[3 * r + 0]));
        s1 = sbox_t<D>(add(s1, ter[3 * r + 1]));
        s2 = sbox_t<D>(add(s2, ter[3 * r + 2]));
        if (lin)
            ext_layer_gen_t(s0, s1, s2, lin);
        else
            ext_layer_t(s0, s1, s2);
    }
}

__attribute__((target("avx512f,avx512ifma"))) void rc_to_ifma(const Fr* rc, size_t n, std::vector<Lane8>& out) {
    static_assert(sizeof(V) == 5 * sizeof(Lane8), "V is 5 limbs of 8 lanes");
    out.assign(n * 5, Lane8{});
    for (size_t i = 0; i < n; ++i) {
        const V v = load(rc + i, 0, 8);  // stride 0: the constant in every lane
        std::memcpy(&out[5 * i], &v, sizeof(V));
    }
}

// the generic layers' constants, after the round constants (poseidon2.hpp)
inline const V* lin_ptr(const V* rc, const P2Layout& L) { return L.gen_lin ? rc + p2_lin_offset(L) : nullptr; }

template <uint32_t D>
__attribute__((target("avx512f,avx512ifma"))) void compress8_t(const Fr* left, const Fr* right, size_t stride,
                                                                Fr* out, int n, const V* rc, const P2Layout& L) {
    V s0 = load(left, stride, n), s1 = load(right, stride, n), s2;
    for (int k = 0; k < 5; ++k) s2.l[k] = _mm512_setzero_si512();
    permute<D>(s0, s1, s2, rc, L.rounds_f, L.rounds_p, lin_ptr(rc, L));
    store(s0, out, 1, n);
}

template <uint32_t D>
__attribute__((target("avx512f,avx512ifma"))) void compress16_t(const Fr* left, const Fr* right, size_t stride,
                                                                 Fr* out, int n, const V* rc, const P2Layout& L) {
    const int n1 = n < 8 ? n : 8, n2 = n - n1;
    W s0{load(left, stride, n1), load(left + 8 * stride, stride, n2)};
    W s1{load(right, stride, n1), load(right + 8 * stride, stride, n2)};
    W s2;
    for (int k = 0; k < 5; ++k) s2.x.l[k] = s2.y.l[k] = _mm512_setzero_si512();
    permute<D>(s0, s1, s2, rc, L.rounds_f, L.rounds_p, lin_ptr(rc, L));
    store(s0.x, out, 1, n1);
    store(s0.y, out + 8, 1, n2);
}

template <uint32_t D>
__attribute__((target("avx512f,avx512ifma"))) void hash8_t(const Fr* rows, size_t w, Fr* out, int n, const V* rc,
                                                            const P2Layout& L) {
    V s0, s1, s2;
    for (int k = 0; k < 5; ++k) s0.l[k] = s1.l[k] = s2.l[k] = _mm512_setzero_si512();
    size_t k = 0;
    while (k + 2 <= w) {
        s0 = load(rows + k, w, n);
        s1 = load(rows + k + 1, w, n);
        permute<D>(s0, s1, s2, rc, L.rounds_f, L.rounds_p, lin_ptr(rc, L));
        k += 2;
    }
    if (k < w) {
        s0 = load(rows + k, w, n);
        permute<D>(s0, s1, s2, rc, L.rounds_f, L.rounds_p, lin_ptr(rc, L));
    }
    store(s0, out, 1, n);
}

const V* rc_ptr(const std::vector<Lane8>& v) { return reinterpret_cast<const V*>(v.data()); }
}  // namespace

bool available() {
    static const bool ok = [] {
        if (const char* e = std::getenv("LSP_HOST_IFMA"))
            if (std::atoi(e) == 0) return false;
        __builtin_cpu_init();
        return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512ifma");
    }();
    return ok;
}

void prepare(const std::vector<Fr>& rc, std::vector<Lane8>& out) { rc_to_ifma(rc.data(), rc.size(), out); }

void compress8(const Fr* left, const Fr* right, size_t stride, Fr* out, int n, const std::vector<Lane8>& rc,
               const P2Layout& L) {
    if (L.sbox_degree == 17)
        compress8_t<17>(left, right, stride, out, n, rc_ptr(rc), L);
    else
        compress8_t<11>(left, right, stride, out, n, rc_ptr(rc), L);
}

void compress16(const Fr* left, const Fr* right, size_t stride, Fr* out, int n, const std::vector<Lane8>& rc,
                const P2Layout& L) {
    if (L.sbox_degree == 17)
        compress16_t<17>(left, right, stride, out, n, rc_ptr(rc), L);
    else
        compress16_t<11>(left, right, stride, out, n, rc_ptr(rc), L);
}

void hash8(const Fr* rows, size_t w, Fr* out, int n, const std::vector<Lane8>& rc, const P2Layout& L) {
    if (L.sbox_degree == 17)
        hash8_t<17>(rows, w, out, n, rc_ptr(rc), L);
    else
        hash8_t<11>(rows, w, out, n, rc_ptr(rc), L);
}

}  // namespace ifma
}  // namespace lsp
#endif  // __HIP_DEVICE_COMPILE__
