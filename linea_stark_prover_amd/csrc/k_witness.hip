// Witness generation on the device: the trace crate's
// RawPermutationTrace::get_trace (trace/src/permutation.rs:24-93) and
// RawLookupTrace::get_trace (trace/src/lookup.rs:46-176), writing the
// columns straight into the row-major trace of RawTrace::get_trace
// (trace/src/lib.rs:94-106).  Every kernel here is hand-written:
//
//   rows         one thread per row: copy the raw columns into the trace row,
//                Horner row combinations sum_j c_j alpha^(k-1-j)
//   inverses     launch_batch_inverse (k_field.hip)
//   scans        the permutation check column is a prefix PRODUCT
//                (trace/src/permutation.rs:72), the LogUp column a prefix SUM
//                (trace/src/lookup.rs:152-160): a reduce-then-scan over
//                2048-element tiles (tile aggregates up, their scan, then each
//                tile rescanned from its prefix), recursive over the aggregates
//   multiplicity LogUp's occurrence map (trace/src/lookup.rs:78-100,145-155: a
//                HashMap keyed by the A row combination, counted over the
//                enabled A rows, each entry consumed by the first enabled B
//                entry with the same key in (row, table) order) as a device
//                hash table keyed by the combination: enabled A rows add 1 to
//                their key's count, enabled B entries atomicMin their (row,
//                table) position into it; the B entry holding the minimum
//                receives the count.  Sums and minima do not depend on the
//                order the threads run in, so the result is deterministic.
#include <algorithm>

#include "k_common.hpp"
#include "kernels.hpp"

namespace lsp {

namespace {
// the scan operators (both commutative and associative in Fr)
struct FrMulOp {
    __device__ Fr operator()(const Fr& a, const Fr& b) const { return fr_mul(a, b); }
    __device__ static Fr identity() { return fr_one(); }
};
struct FrAddOp {
    __device__ Fr operator()(const Fr& a, const Fr& b) const { return fr_add(a, b); }
    __device__ static Fr identity() { return fr_zero(); }
};

// ---- inclusive scan: tiles of SC_PER contiguous elements per thread
constexpr uint32_t SC_THREADS = 256, SC_PER = 8, SC_TILE = SC_THREADS * SC_PER;

// this thread's SC_PER elements of the tile, folded
template <class Op>
__device__ __forceinline__ Fr sc_thread_agg(const Fr* __restrict__ in, size_t n, size_t base, Op op) {
    Fr a = Op::identity();
#pragma unroll
    for (uint32_t j = 0; j < SC_PER; ++j)
        if (base + j < n) a = op(a, in[base + j]);
    return a;
}

// exclusive scan of the block's thread values (Hillis-Steele in LDS); *total = all of them
template <class Op>
__device__ __forceinline__ Fr sc_block_excl(Fr v, Fr* lds, Op op, Fr* total) {
    const uint32_t t = threadIdx.x;
    lds[t] = v;
    __syncthreads();
    for (uint32_t d = 1; d < SC_THREADS; d <<= 1) {
        const Fr x = t >= d ? op(lds[t - d], v) : v;
        __syncthreads();
        lds[t] = x;
        v = x;
        __syncthreads();
    }
    const Fr ex = t ? lds[t - 1] : Op::identity();
    if (total) *total = lds[SC_THREADS - 1];
    return ex;
}

template <class Op>
__global__ __launch_bounds__(SC_THREADS) void k_scan_up(const Fr* __restrict__ in, size_t n, Fr* __restrict__ agg) {
    __shared__ Fr lds[SC_THREADS];
    const Op op;
    const size_t base = (size_t)blockIdx.x * SC_TILE + (size_t)threadIdx.x * SC_PER;
    Fr total;
    sc_block_excl(sc_thread_agg(in, n, base, op), lds, op, &total);
    if (threadIdx.x == 0) agg[blockIdx.x] = total;
}

// incl_agg (nullable): the inclusive scan of the tile aggregates; tile b starts from incl_agg[b - 1]
template <class Op>
__global__ __launch_bounds__(SC_THREADS) void k_scan_down(const Fr* __restrict__ in, Fr* __restrict__ out, size_t n,
                                                          const Fr* __restrict__ incl_agg) {
    __shared__ Fr lds[SC_THREADS];
    const Op op;
    const size_t base = (size_t)blockIdx.x * SC_TILE + (size_t)threadIdx.x * SC_PER;
    Fr pre = sc_block_excl(sc_thread_agg(in, n, base, op), lds, op, nullptr);
    if (incl_agg && blockIdx.x) pre = op(incl_agg[blockIdx.x - 1], pre);
#pragma unroll
    for (uint32_t j = 0; j < SC_PER; ++j) {
        if (base + j >= n) break;
        pre = op(pre, in[base + j]);
        out[base + j] = pre;
    }
}

template <class Op>
hipError_t scan_rec(const Fr* in, Fr* out, size_t n, Fr* scratch, size_t cap, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const size_t T = (n + SC_TILE - 1) / SC_TILE;
    if (T == 1) {
        hipLaunchKernelGGL(k_scan_down<Op>, dim3(1), dim3(SC_THREADS), 0, st, in, out, n, nullptr);
        return hipGetLastError();
    }
    if (2 * T > cap) return hipErrorInvalidValue;
    Fr* agg = scratch;
    Fr* agg_incl = scratch + T;
    hipLaunchKernelGGL(k_scan_up<Op>, dim3((unsigned)T), dim3(SC_THREADS), 0, st, in, n, agg);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = scan_rec<Op>(agg, agg_incl, T, scratch + 2 * T, cap - 2 * T, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_scan_down<Op>, dim3((unsigned)T), dim3(SC_THREADS), 0, st, in, out, n, agg_incl);
    return hipGetLastError();
}

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

// ---- LogUp occurrences: a device hash table over the row combinations.
// Record r: r < n -> A row r, key comb[r]; else B entry (t, i) with
// r = n + t n + i, key comb[r] (comb is [A | table 0 | table 1 | ...]).
constexpr uint32_t H_EMPTY = 0xffffffffu;

__device__ __forceinline__ uint32_t key_hash(const Fr& k) {
    uint64_t x = ((uint64_t)k.v[1] << 32 | k.v[0]) ^ (((uint64_t)k.v[5] << 32 | k.v[4]) * 0x9E3779B97F4A7C15ull);
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    return (uint32_t)(x ^ (x >> 32));
}

__device__ __forceinline__ bool rec_enabled(uint32_t r, size_t n, const Fr* afil, const Fr* bfil) {
    return r < n ? fr_nonzero(afil[r]) : fr_nonzero(bfil[r - n]);
}

// the slot of comb[r]'s key (linear probing; insert claims an empty slot
// with a CAS -- slots never change once claimed, so every thread with the
// same key ends in the same slot).  Without insert the key is looked up: an
// empty slot ends the probe (H_EMPTY, absent).  Every probe ends within the
// table's mask + 1 slots: the table has at least twice as many slots as
// records (occ_capacity), and a full sweep returns H_EMPTY rather than spin.
__device__ __forceinline__ uint32_t occ_slot(const Fr* __restrict__ comb, uint32_t r, uint32_t* rep, uint32_t mask,
                                             bool insert, size_t m) {
    const Fr key = comb[r];
    uint32_t h = key_hash(key) & mask;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        uint32_t cur = __hip_atomic_load(rep + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == H_EMPTY) {
            if (!insert) return H_EMPTY;
            cur = atomicCAS(rep + h, H_EMPTY, r);
            if (cur == H_EMPTY) return h;
        }
        if (!LSP_BOUNDS(cur < m)) return H_EMPTY;  // a slot holds a record index below m
        if (cur == r || fr_eq(comb[cur], key)) return h;
        h = (h + 1) & mask;
    }
    return H_EMPTY;
}

// enabled A rows count their key; enabled B entries record their (row, table)
// position i nt + t, the order the reference's loop meets them in
__global__ __launch_bounds__(256) void k_occ_insert(const Fr* __restrict__ comb, size_t n, uint32_t nt,
                                                    const Fr* __restrict__ afil, const Fr* __restrict__ bfil, size_t m,
                                                    uint32_t* rep, uint32_t* cnt, unsigned long long* minb,
                                                    uint32_t mask) {
    const size_t r = gtid();
    if (r >= m || !rec_enabled((uint32_t)r, n, afil, bfil)) return;
    const uint32_t h = occ_slot(comb, (uint32_t)r, rep, mask, true, m);
    if (h == H_EMPTY) return;  // (a full table: excluded by occ_capacity)
    if (r < n) {
        atomicAdd(cnt + h, 1u);
    } else {
        const size_t t = (r - n) / n, i = (r - n) - t * n;
        atomicMin(minb + h, (unsigned long long)(i * nt + t));
    }
}

// the first enabled B entry of each key takes the key's count of enabled A rows
__global__ __launch_bounds__(256) void k_occ_assign(const Fr* __restrict__ comb, size_t n, uint32_t nt,
                                                    const Fr* __restrict__ bfil, uint32_t* rep,
                                                    const uint32_t* __restrict__ cnt,
                                                    const unsigned long long* __restrict__ minb, uint32_t mask,
                                                    uint32_t* __restrict__ occ) {
    const size_t j = gtid();  // B entry t n + i
    if (j >= n * nt || !fr_nonzero(bfil[j])) return;
    const uint32_t h = occ_slot(comb, (uint32_t)(n + j), rep, mask, false, n * (nt + 1));
    if (h == H_EMPTY) return;  // (every enabled B entry was inserted by k_occ_insert)
    if (!LSP_BOUNDS(h <= mask)) return;
    const size_t t = j / n, i = j - t * n;
    if (minb[h] == (unsigned long long)(i * nt + t)) occ[j] = cnt[h];
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

// the occurrence table's capacity: a power of two >= 2 records (load <= 1/2)
static size_t occ_capacity(size_t m) {
    size_t c = 64;
    while (c < 2 * m) c <<= 1;
    return c;
}

size_t witness_scratch_bytes(size_t n, uint32_t nt) {
    // the occurrence table (4 + 4 + 8 bytes per slot) or the scans' tile
    // aggregates (2 per tile, every level), whichever a block needs
    const size_t m = n * (1 + (size_t)nt);
    const size_t table = occ_capacity(m) * 16 + 3 * 256;
    const size_t scan = (2 * (n / SC_TILE + 1) + 64) * sizeof(Fr) * 2;
    return std::max(table, scan);
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
    Fr* s = (Fr*)scratch;
    const size_t cap = scratch_bytes / sizeof(Fr);
    return product ? scan_rec<FrMulOp>(in, out, n, s, cap, st) : scan_rec<FrAddOp>(in, out, n, s, cap, st);
}

hipError_t launch_lookup_occurrences(const Fr* comb, size_t n, uint32_t nt, const Fr* afil, const Fr* bfil,
                                     uint32_t* occ, void* scratch, size_t scratch_bytes, hipStream_t st) {
    const size_t m = n * (1 + (size_t)nt);
    // record ids are 32-bit and slot ids must stay below H_EMPTY: <= 2^30 records
    // (a table of <= 2^31 slots)
    if (m > (1ull << 30)) return hipErrorInvalidValue;
    const size_t cap = occ_capacity(m);
    char* p = (char*)scratch;
    auto* minb = (unsigned long long*)p;  // 8-byte entries first (alignment)
    auto* rep = (uint32_t*)(p + cap * 8);
    auto* cnt = rep + cap;
    if (cap * 16 > scratch_bytes) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(minb, 0xff, cap * 8, st);
    if (e == hipSuccess) e = hipMemsetAsync(rep, 0xff, cap * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, cap * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(occ, 0, n * nt * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    const uint32_t mask = (uint32_t)(cap - 1);
    hipLaunchKernelGGL(k_occ_insert, dim3(nblocks(m, 256)), dim3(256), 0, st, comb, n, nt, afil, bfil, m, rep, cnt,
                       minb, mask);
    if (nt)
        hipLaunchKernelGGL(k_occ_assign, dim3(nblocks(n * nt, 256)), dim3(256), 0, st, comb, n, nt, bfil, rep, cnt, minb,
                           mask, occ);
    return hipGetLastError();
}

hipError_t launch_lookup_terms(const Fr* inv, const uint32_t* occ, const Fr* afil, size_t n, uint32_t nt, Fr* out,
                               size_t ostride, uint32_t col_ainv, Fr* term, hipStream_t st) {
    hipLaunchKernelGGL(k_lookup_terms, dim3(nblocks(n, 256)), dim3(256), 0, st, inv, occ, afil, n, nt, out, ostride,
                       col_ainv, term);
    return hipGetLastError();
}

}  // namespace lsp

LSP_BOUNDS_READER(k_witness)
