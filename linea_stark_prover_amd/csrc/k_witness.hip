// Witness generation on the device: the trace crate's
// RawPermutationTrace::get_trace (trace/src/permutation.rs:24-93) and
// RawLookupTrace::get_trace (trace/src/lookup.rs:46-176), writing the
// columns straight into the row-major trace of RawTrace::get_trace
// (trace/src/lib.rs:94-106).
//
//   rows         one thread per row: copy the raw columns into the trace row,
//                Horner row combinations sum_j c_j alpha^(k-1-j)
//   inverses     launch_batch_inverse (k_field.hip)
//   scans        the permutation check column is a prefix PRODUCT, the LogUp
//                column a prefix SUM: hipCUB decoupled-lookback scans over Fr
//   multiplicity LogUp's occurrence map (a HashMap keyed by the A row
//                combination, entries consumed by the first enabled B row with
//                the same key, row-major over (row, table)) as a stable LSD
//                radix sort of every entry on (key, tag, position): in each
//                run of equal keys the enabled A entries come first, so the
//                first enabled B entry of the run receives the run's A count.
#include <hipcub/hipcub.hpp>

#include "k_common.hpp"
#include "kernels.hpp"

namespace lsp {

namespace {
struct FrMulOp {
    __device__ Fr operator()(const Fr& a, const Fr& b) const { return fr_mul(a, b); }
};
struct FrAddOp {
    __device__ Fr operator()(const Fr& a, const Fr& b) const { return fr_add(a, b); }
};

__device__ __forceinline__ bool fr_nonzero(const Fr& x) {
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) o |= x.v[k];
    return o != 0;
}

__global__ __launch_bounds__(256) void k_perm_rows(const Fr* __restrict__ a, uint32_t na, const Fr* __restrict__ b,
                                                   uint32_t nb, size_t n, Fr alpha, Fr delta, Fr* __restrict__ out,
                                                   size_t ostride, Fr* __restrict__ al, Fr* __restrict__ bl) {
    const size_t i = gtid();
    if (i >= n) return;
    Fr* row = out + i * ostride;
    Fr acc = fr_zero();
    for (uint32_t k = 0; k < na; ++k) {
        const Fr v = a[k * n + i];
        row[k] = v;
        acc = fr_add(fr_mul(acc, alpha), v);
    }
    al[i] = fr_add(acc, delta);
    acc = fr_zero();
    for (uint32_t k = 0; k < nb; ++k) {
        const Fr v = b[k * n + i];
        row[na + k] = v;
        acc = fr_add(fr_mul(acc, alpha), v);
    }
    bl[i] = fr_add(acc, delta);
}

// comb[0][i] = A row combination, comb[1+t][i] = table t's; den = comb + delta
__global__ __launch_bounds__(256) void k_lookup_rows(const Fr* __restrict__ a, uint32_t na, const Fr* __restrict__ b,
                                                     uint32_t nt, uint32_t nbc, const Fr* __restrict__ afil,
                                                     const Fr* __restrict__ bfil, size_t n, Fr alpha, Fr delta,
                                                     Fr* __restrict__ out, size_t ostride, Fr* __restrict__ comb,
                                                     Fr* __restrict__ den) {
    const size_t i = gtid();
    if (i >= n) return;
    Fr* row = out + i * ostride;
    Fr acc = fr_zero();
    for (uint32_t k = 0; k < na; ++k) {
        const Fr v = a[k * n + i];
        row[k] = v;
        acc = fr_add(fr_mul(acc, alpha), v);
    }
    comb[i] = acc;
    den[i] = fr_add(acc, delta);
    for (uint32_t t = 0; t < nt; ++t) {
        acc = fr_zero();
        for (uint32_t k = 0; k < nbc; ++k) {
            const Fr v = b[((size_t)t * nbc + k) * n + i];
            row[na + t * nbc + k] = v;
            acc = fr_add(fr_mul(acc, alpha), v);
        }
        comb[(1 + (size_t)t) * n + i] = acc;
        den[(1 + (size_t)t) * n + i] = fr_add(acc, delta);
    }
    const uint32_t f0 = na + nt * nbc;
    row[f0] = afil[i];
    for (uint32_t t = 0; t < nt; ++t) row[f0 + 1 + t] = bfil[(size_t)t * n + i];
}

// sort record r: r < n -> A row r; else B entry (t, i) = ((r-n)/n, (r-n)%n).
// tag 0 = enabled A, 1 = enabled B, 2 = disabled (sorts after both)
__device__ __forceinline__ uint64_t rec_tagpos(uint32_t r, size_t n, uint32_t nt, const Fr* afil, const Fr* bfil) {
    if (r < n) return (fr_nonzero(afil[r]) ? 0ull : 2ull) << 40 | r;
    const size_t t = (r - n) / n, i = (r - n) % n;
    const uint64_t tag = fr_nonzero(bfil[t * n + i]) ? 1ull : 2ull;
    return tag << 40 | (i * nt + t);
}

// pass 0: tag/position; pass 1..4: 64-bit word (pass-1) of the key
__global__ __launch_bounds__(256) void k_sort_keys(const uint32_t* __restrict__ perm, size_t m, int pass,
                                                   const Fr* __restrict__ comb, size_t n, uint32_t nt,
                                                   const Fr* __restrict__ afil, const Fr* __restrict__ bfil,
                                                   uint64_t* __restrict__ keys) {
    const size_t j = gtid();
    if (j >= m) return;
    const uint32_t r = perm[j];
    if (pass == 0) {
        keys[j] = rec_tagpos(r, n, nt, afil, bfil);
    } else {
        const Fr& k = comb[r];
        const int w = pass - 1;
        keys[j] = (uint64_t)k.v[2 * w] | ((uint64_t)k.v[2 * w + 1] << 32);
    }
}

__global__ __launch_bounds__(256) void k_iota(uint32_t* __restrict__ p, size_t m) {
    const size_t j = gtid();
    if (j < m) p[j] = (uint32_t)j;
}

// run_start[j] = j if sorted record j starts a run of equal keys, else 0
__global__ __launch_bounds__(256) void k_run_starts(const uint32_t* __restrict__ perm, size_t m,
                                                    const Fr* __restrict__ comb, uint64_t* __restrict__ rs) {
    const size_t j = gtid();
    if (j >= m) return;
    rs[j] = (j == 0 || !fr_eq(comb[perm[j]], comb[perm[j - 1]])) ? j : 0;
}

// the first enabled B entry of each run gets the run's count of enabled A entries
__global__ __launch_bounds__(256) void k_first_b(const uint32_t* __restrict__ perm, size_t m, const uint64_t* rs,
                                                 size_t n, uint32_t nt, const Fr* __restrict__ afil,
                                                 const Fr* __restrict__ bfil, uint32_t* __restrict__ occ) {
    const size_t j = gtid();
    if (j >= m) return;
    const uint32_t r = perm[j];
    if ((rec_tagpos(r, n, nt, afil, bfil) >> 40) != 1) return;
    const size_t s = rs[j];
    if (j != s && (rec_tagpos(perm[j - 1], n, nt, afil, bfil) >> 40) == 1) return;  // not the first B of its run
    // records s .. j-1 of the run are its enabled A entries (tag 0 sorts first)
    occ[r - n] = (uint32_t)(j - s);
}

// term[i] = [a_filter != 0] a_inv[i] - sum_t occ[t][i] b_inv[t][i]; writes the
// a_inverses, b_inverses and multiplicities columns
__global__ __launch_bounds__(256) void k_lookup_terms(const Fr* __restrict__ inv, const uint32_t* __restrict__ occ,
                                                      const Fr* __restrict__ afil, size_t n, uint32_t nt,
                                                      Fr* __restrict__ out, size_t ostride, uint32_t col_ainv,
                                                      Fr* __restrict__ term) {
    const size_t i = gtid();
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

__global__ __launch_bounds__(256) void k_mul_vec(const Fr* __restrict__ x, const Fr* __restrict__ y, size_t n,
                                                 Fr* __restrict__ out) {
    const size_t i = gtid();
    if (i < n) out[i] = fr_mul(x[i], y[i]);
}

__global__ __launch_bounds__(256) void k_put_col(const Fr* __restrict__ v, size_t n, Fr* __restrict__ out,
                                                 size_t ostride, uint32_t col) {
    const size_t i = gtid();
    if (i < n) out[i * ostride + col] = v[i];
}

// hipCUB temp storage in a caller scratch region
struct Scratch {
    void* p;
    size_t cap;
};
template <class F>
hipError_t with_temp(Scratch s, F&& f) {
    size_t need = 0;
    hipError_t e = f(nullptr, need);
    if (e != hipSuccess) return e;
    if (need > s.cap) return hipErrorInvalidValue;
    return f(s.p, need);
}

// Synthetic raw permutation columns generated on the device (bench inputs at
// sizes where a host generator would hold tens of GiB per rank): a[c][i] is a
// counter-based hash of (seed, c, i) masked to 252 bits (< r), in Montgomery
// form; b[c][i] = a[c][pi(i)] with the row bijection pi(i) = (mul i + add)
// mod n (mul odd), the same for every column -- B is a row shuffle of A, as
// the permutation argument requires.  Deterministic in the seed, so every
// rank of a sharded proof builds the same trace without moving it.
__device__ __forceinline__ uint64_t smix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ Fr gen_value(uint64_t seed, uint32_t c, size_t i) {
    Fr x;
    const uint64_t base = seed * 0x9E3779B97F4A7C15ull + ((uint64_t)c << 40) + ((uint64_t)i << 2);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t v = smix(base + (uint64_t)k + 0x632BE59BD9B4E019ull);
        x.v[2 * k] = (uint32_t)v;
        x.v[2 * k + 1] = (uint32_t)(v >> 32);
    }
    x.v[7] &= (1u << 28) - 1;  // < 2^252 < r
    return fr_mul(x, fr_r2());
}
__global__ __launch_bounds__(256) void k_gen_raw_perm(uint64_t seed, size_t n, uint32_t ncols, uint64_t mul,
                                                      uint64_t add, Fr* __restrict__ a, Fr* __restrict__ b) {
    const size_t i = gtid();
    if (i >= n) return;
    const size_t j = (size_t)((mul * (uint64_t)i + add) & (uint64_t)(n - 1));
    for (uint32_t c = 0; c < ncols; ++c) {
        a[c * n + i] = gen_value(seed, c, i);
        b[c * n + i] = gen_value(seed, c, j);
    }
}
}  // namespace

size_t witness_scratch_bytes(size_t n, uint32_t nt) {
    // sort keys/perms (double buffered) + run starts + hipCUB temp (generous bound)
    const size_t m = n * (1 + (size_t)nt);
    return m * (2 * sizeof(uint64_t) + 2 * sizeof(uint32_t) + 2 * sizeof(uint64_t)) + 6 * 256 + (64u << 20) + m * 64;
}

hipError_t launch_gen_raw_perm(uint64_t seed, size_t n, uint32_t ncols, uint64_t mul, uint64_t add, Fr* a, Fr* b,
                               hipStream_t st) {
    hipLaunchKernelGGL(k_gen_raw_perm, dim3(nblocks(n, 256)), dim3(256), 0, st, seed, n, ncols, mul, add, a, b);
    return hipGetLastError();
}

hipError_t launch_perm_rows(const Fr* a, uint32_t na, const Fr* b, uint32_t nb, size_t n, Fr alpha, Fr delta,
                            Fr* out, size_t ostride, Fr* al, Fr* bl, hipStream_t st) {
    hipLaunchKernelGGL(k_perm_rows, dim3(nblocks(n, 256)), dim3(256), 0, st, a, na, b, nb, n, alpha, delta, out,
                       ostride, al, bl);
    return hipGetLastError();
}

hipError_t launch_lookup_rows(const Fr* a, uint32_t na, const Fr* b, uint32_t nt, uint32_t nbc, const Fr* afil,
                              const Fr* bfil, size_t n, Fr alpha, Fr delta, Fr* out, size_t ostride, Fr* comb,
                              Fr* den, hipStream_t st) {
    hipLaunchKernelGGL(k_lookup_rows, dim3(nblocks(n, 256)), dim3(256), 0, st, a, na, b, nt, nbc, afil, bfil, n, alpha,
                       delta, out, ostride, comb, den);
    return hipGetLastError();
}

hipError_t launch_mul_vec(const Fr* x, const Fr* y, size_t n, Fr* out, hipStream_t st) {
    hipLaunchKernelGGL(k_mul_vec, dim3(nblocks(n, 256)), dim3(256), 0, st, x, y, n, out);
    return hipGetLastError();
}

hipError_t launch_put_col(const Fr* v, size_t n, Fr* out, size_t ostride, uint32_t col, hipStream_t st) {
    hipLaunchKernelGGL(k_put_col, dim3(nblocks(n, 256)), dim3(256), 0, st, v, n, out, ostride, col);
    return hipGetLastError();
}

hipError_t launch_fr_scan(const Fr* in, Fr* out, size_t n, bool product, void* scratch, size_t scratch_bytes,
                          hipStream_t st) {
    Scratch s{scratch, scratch_bytes};
    if (product)
        return with_temp(s, [&](void* p, size_t& b) {
            return hipcub::DeviceScan::InclusiveScan(p, b, in, out, FrMulOp(), (int)n, st);
        });
    return with_temp(s, [&](void* p, size_t& b) {
        return hipcub::DeviceScan::InclusiveScan(p, b, in, out, FrAddOp(), (int)n, st);
    });
}

hipError_t launch_lookup_occurrences(const Fr* comb, size_t n, uint32_t nt, const Fr* afil, const Fr* bfil,
                                     uint32_t* occ, void* scratch, size_t scratch_bytes, hipStream_t st) {
    const size_t m = n * (1 + (size_t)nt);
    // every partition 256-byte aligned (hipCUB's temp storage expects it)
    char* p = (char*)scratch;
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        char* q = p + off;
        off += (bytes + 255) & ~(size_t)255;
        return q;
    };
    uint64_t* k0 = (uint64_t*)carve(m * 8);
    uint64_t* k1 = (uint64_t*)carve(m * 8);
    uint32_t* p0 = (uint32_t*)carve(m * 4);
    uint32_t* p1 = (uint32_t*)carve(m * 4);
    uint64_t* rs = (uint64_t*)carve(m * 8);
    uint64_t* rs2 = (uint64_t*)carve(m * 8);
    char* tmp = p + off;
    const size_t used = off;
    if (used > scratch_bytes) return hipErrorInvalidValue;
    Scratch s{tmp, scratch_bytes - used};
    const unsigned g = nblocks(m, 256);
    hipLaunchKernelGGL(k_iota, dim3(g), dim3(256), 0, st, p0, m);
    for (int pass = 0; pass < 5; ++pass) {
        hipLaunchKernelGGL(k_sort_keys, dim3(g), dim3(256), 0, st, p0, m, pass, comb, n, nt, afil, bfil, k0);
        const int end_bit = pass == 0 ? 42 : 64;
        hipError_t e = with_temp(s, [&](void* t, size_t& b) {
            return hipcub::DeviceRadixSort::SortPairs(t, b, k0, k1, p0, p1, (int)m, 0, end_bit, st);
        });
        if (e != hipSuccess) return e;
        std::swap(p0, p1);
    }
    hipLaunchKernelGGL(k_run_starts, dim3(g), dim3(256), 0, st, p0, m, comb, rs);
    hipError_t e = with_temp(s, [&](void* t, size_t& b) {
        return hipcub::DeviceScan::InclusiveScan(t, b, rs, rs2, hipcub::Max(), (int)m, st);
    });
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(occ, 0, n * nt * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_first_b, dim3(g), dim3(256), 0, st, p0, m, rs2, n, nt, afil, bfil, occ);
    return hipGetLastError();
}

hipError_t launch_lookup_terms(const Fr* inv, const uint32_t* occ, const Fr* afil, size_t n, uint32_t nt, Fr* out,
                               size_t ostride, uint32_t col_ainv, Fr* term, hipStream_t st) {
    hipLaunchKernelGGL(k_lookup_terms, dim3(nblocks(n, 256)), dim3(256), 0, st, inv, occ, afil, n, nt, out, ostride,
                       col_ainv, term);
    return hipGetLastError();
}

}  // namespace lsp
