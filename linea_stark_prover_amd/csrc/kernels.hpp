// Device kernels of the hot path and their host launchers.
// Each launcher enqueues on `st` and returns hipError_t of the launch.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "fr.hpp"
#include "fr29.hpp"
#include "poseidon2.hpp"

namespace lsp {

// ------------------------------------------------------------ k_ntt.hip
// Where column c of a transform sits in its source matrix.
//   plain    element (row, c) at row * stride + c0 + cstep * c; source
//            columns >= valid read as zero (a rank's strided column subset)
//   blocked  the column-split layout of a sharded proof's coefficients: G =
//            2^logb row-major blocks of h x bw, column c in block
//            bitrev_logb(c mod G) at column c / G (rank g inverted the columns
//            bitrev(g) + G k, and the blocks arrive in rank order)
constexpr uint32_t COLMAP_PLAIN = 0xffu;
struct ColMap {
    uint32_t logb = COLMAP_PLAIN;
    uint32_t stride = 0, c0 = 0, cstep = 1, valid = 0xffffffffu;
    uint32_t bw = 0;
    static ColMap plain(uint32_t w) {
        ColMap m;
        m.stride = w;
        m.valid = w;
        return m;
    }
    static ColMap blocked(uint32_t logb, uint32_t bw) {
        ColMap m;
        m.logb = logb;
        m.bw = bw;
        return m;
    }
};
// Coset evaluations of the h x w row-major matrix `in`: `ncosets` blocks of h
// rows (block k on the coset of twist table k), each in bit-reversed order,
// into row-major `out` (canonical), via X (h x w scratch, left holding
// h * coefficients reduced below 2r).  tw_inv / tw_fwd: w_h^-x / w_h^x, x < h/2;
// twist: two-level tables (L1, L2) of base s and scale 1/h, one per coset
// (twist_per_col = 0) or per (coset, column) at index k*w + c -- all tables in
// the 29-bit Montgomery form (launch_to_f29form; k_ntt.hip).  ratio (nullptr:
// off; ncosets a power of two >= 2): the two-level table (L1, L2) of rho^i when
// the shifts of blocks bitrev(0), bitrev(1), ... are s, s rho, s rho^2, ...; the
// fused pass then uses only block 0's twist tables and chains the rest.
hipError_t launch_lde(const Fr* in, Fr* X, Fr* out, size_t w, uint32_t logh, uint32_t ncosets, const uint4* tw_inv,
                      const uint4* tw_fwd, const Fr* twist, uint32_t L1, uint32_t L2, int twist_per_col,
                      const Fr* ratio, hipStream_t st);
// The two halves of launch_lde, for a sharded proof whose ranks split the
// inverse transform by columns (prove.cpp prove_shard):
//   launch_intt       X (h x w) <- h * coefficients, natural order, of the w
//                     columns `map` picks in `in` (values on H_h)
//   launch_lde_coeffs the coset blocks of launch_lde from h * coefficients at
//                     `coef` through `map` (no inverse stages)
hipError_t launch_intt(const Fr* in, ColMap map, Fr* X, size_t w, uint32_t logh, const uint4* tw_inv, hipStream_t st);
hipError_t launch_lde_coeffs(const Fr* coef, ColMap map, Fr* out, size_t w, uint32_t logh, uint32_t ncosets,
                             const uint4* tw_fwd, const Fr* twist, uint32_t L1, uint32_t L2, int twist_per_col,
                             const Fr* ratio, hipStream_t st);
// A sub-coset of the LDE (a sharded proof over more ranks than cosets):
// out (S x w, row-major) = the h coefficients of every column folded to S,
// out[i][c] = sum_t coef[i + t S][c] fac[c f + t] for t < f = h / S (coef read
// through `map`, values as launch_intt leaves them; fac: the f factors
// sigma_c^t / f of each column in the 29-bit form, launch_to_f29form).  The
// size-S coset NTT of the folded column equals the degree < h polynomial on
// that size-S coset when sigma_c = (its shift)^S.
hipError_t launch_fold_subcoset(const Fr* coef, ColMap map, size_t h, size_t S, uint32_t w, const Fr* fac, Fr* out,
                                hipStream_t st);
// ark-form words -> the 29-bit Montgomery form (x 2^261 mod r), canonical, in place allowed
hipError_t launch_to_f29form(const Fr* in, Fr* out, size_t n, hipStream_t st);
// out[i][c] = X[i][c] * f^i, canonical; tab: two-level table of f in the 29-bit form (k_scale_coeffs)
hipError_t launch_scale_coeffs(const Fr* X, size_t h, uint32_t w, const Fr* tab, uint32_t L1, Fr* out,
                               hipStream_t st);
// the same, unpacked into 9 x 29-bit limbs padded to 48 bytes (3 x uint4 per
// element): the NTT's twiddle tables, loaded with no repacking
hipError_t launch_to_f29limbs(const Fr* in, uint4* out, size_t n, hipStream_t st);
// stage-major twiddles for k_ntt_rm: entry 2^(m-1) - 1 + i = w_(2^m)^i (i < 2^(m-1),
// m = 1..logH) from pw[x] = w_H^x (x < H/2), in the 48-byte 29-bit-limb slots
hipError_t launch_stage_twiddles(const Fr* pw, uint32_t logH, uint4* out, hipStream_t st);
// Two-level power tables: for each base b,
// tab[b] = {b^j, j < 2^L1} ++ {b^(j 2^L1) * scale[b], j < 2^L2}   (scale nullable)
hipError_t launch_pow_tables(const Fr* bases, size_t nbases, uint32_t L1, uint32_t L2, const Fr* scale,
                             Fr* tabs, hipStream_t st);
// out[i] = base^i for i < n, from a two-level table of base
hipError_t launch_powers(const Fr* tab, uint32_t L1, size_t n, Fr* out, hipStream_t st);

// ----------------------------------------------------------- k_hash.hip
struct MatList {
    const Fr* ptr[8];
    uint32_t width[8];
    uint32_t n;
};
// round constants (ark form) -> the 29-bit-limb form the permutation kernels take
hipError_t launch_rc_to_f29(const Fr* rc, F29* rc29, uint32_t n, hipStream_t st);
hipError_t launch_permute(Fr* states, size_t n, const F29* rc29, P2Layout L, hipStream_t st);
// out[i] = hash_iter(concat of row i of every matrix in `m`)
// FRI fold of the previous round fused into this round's leaf hashing: the
// folded vector v' (2 n values) is written to `vout` and leaf j = hash_iter(
// v'[2j], v'[2j+1]) to `out`, with v'[i] = (half + p_i) v[2i] + (half - p_i) v[2i+1],
// p_i = half_beta * tab^bitrev_logm(i0 + i) (launch_fri_fold's formula)
struct FoldSpec {
    const Fr* v;      // the previous round's vector (this rank's slice)
    Fr* vout;         // where the folded vector goes
    Fr half, half_beta;
    const Fr* tab;    // two-level table of w_{2M}^-1
    uint32_t L1, logm;
    uint64_t i0;
};
hipError_t launch_fold_hash(const FoldSpec& f, size_t nleaves, Fr* out, const F29* rc, P2Layout L, hipStream_t st);
hipError_t launch_hash_rows(const MatList& m, size_t nrows, Fr* out, const F29* rc29, P2Layout L, hipStream_t st);
// dst[i] = compress(src[2i], src[2i+1]) for i < nout
hipError_t launch_merkle_level(const Fr* src, Fr* dst, size_t nout, const F29* rc29, P2Layout L, hipStream_t st);
// PoW grinding: test witnesses [base, base+count); *best = min hit (caller inits to ~0);
// mont: sample_bits from the Montgomery form (U8)
hipError_t launch_grind(const Fr pre[3], uint32_t wlane, uint64_t base, uint64_t count, uint32_t bits, bool mont,
                        const F29* rc29, P2Layout L, unsigned long long* best, hipStream_t st);
// full tree above the leaf digests already stored at layers[0..nleaves)
hipError_t launch_merkle_tree(Fr* layers, size_t nleaves, const F29* rc29, P2Layout L, hipStream_t st);
// the levels above the leaves while the current layer is longer than stop_len;
// *off_out / *len_out = offset and length of the last layer written
hipError_t launch_merkle_levels(Fr* layers, size_t nleaves, size_t stop_len, const F29* rc29, P2Layout L,
                                size_t* off_out, size_t* len_out, hipStream_t st);

// --------------------------------------------------------- k_field.hip
// out[i] = 1 / in[i] (Montgomery trick, interleaved chunks); in may alias out? no
// out[i] = 1/in[i] (0 -> 0); out != in.  scratch: batch_inverse_scratch(n)
// elements (hierarchical, one Fermat inverse per call), or nullptr for the
// single-level kernel (one inverse per 8..256 elements)
size_t batch_inverse_scratch(size_t n);
// inv_total (optional, host value): 1/(product of all n inputs), when the caller
// knows it in closed form -- the hierarchical path then skips its one Fermat
// inversion (used only with a scratch buffer / n <= BI_BASE)
hipError_t launch_batch_inverse(const Fr* in, Fr* out, size_t n, hipStream_t st, Fr* scratch = nullptr,
                                const Fr* inv_total = nullptr);
// Fr-mul throughput probe: nthreads lanes x iters x 4 independent products
hipError_t launch_calib_mul(Fr* out, size_t nthreads, uint32_t iters, hipStream_t st);
// iters chained Poseidon2 permutations per lane, register-resident (k_hash.hip)
hipError_t launch_calib_perm(Fr* out, size_t nthreads, uint32_t iters, const F29* rc, P2Layout L, hipStream_t st);
// out[i] = *ptrs[i]
hipError_t launch_gather(const uint64_t* ptrs, Fr* out, size_t n, hipStream_t st);
// Sharded quotient exchange: stage holds 2^logGq blocks of h x cpr values,
// block r = chunks j = bitrev(r) + (c << logGq), c < cpr; out = the natural
// h x q chunk matrix (q = cpr << logGq), out[k*q + j].
// out[i] = stage[bitrev(i mod Gq) Sq + i / Gq] for i < Q = Gq Sq: the h x q
// quotient matrix (row k, chunk j = point k q + j) from the Gq ranks' slots of
// Sq points each (rank r computed the points bitrev(r) + Gq m)
hipError_t launch_assemble_chunks(const Fr* stage, uint32_t logGq, size_t Sq, Fr* out, hipStream_t st);

// ----------------------------------------------------- k_witness.hip
// (trace crate semantics; see k_witness.hip)
size_t witness_scratch_bytes(size_t n, uint32_t ntables);
// synthetic raw permutation columns (ncols x n each, column-major): a = seeded
// hash values, b[c][i] = a[c][(mul i + add) mod n]; n a power of two, mul odd
hipError_t launch_gen_raw_perm(uint64_t seed, size_t n, uint32_t ncols, uint64_t mul, uint64_t add, Fr* a, Fr* b,
                               hipStream_t st);
// trace row i (stride ostride): a cols, b cols; al/bl = row combination + delta
hipError_t launch_perm_rows(const Fr* a, uint32_t na, const Fr* b, uint32_t nb, size_t n, Fr alpha, Fr delta,
                            Fr* out, size_t ostride, Fr* al, Fr* bl, hipStream_t st);
// trace row i: a cols, b tables, a_filter, b_filters; comb / den: (1 + nt) x n
hipError_t launch_lookup_rows(const Fr* a, uint32_t na, const Fr* b, uint32_t nt, uint32_t nbc, const Fr* afil,
                              const Fr* bfil, size_t n, Fr alpha, Fr delta, Fr* out, size_t ostride, Fr* comb,
                              Fr* den, hipStream_t st);
hipError_t launch_mul_vec(const Fr* x, const Fr* y, size_t n, Fr* out, hipStream_t st);
hipError_t launch_put_col(const Fr* v, size_t n, Fr* out, size_t ostride, uint32_t col, hipStream_t st);
// inclusive prefix product (product = true) or sum over Fr
hipError_t launch_fr_scan(const Fr* in, Fr* out, size_t n, bool product, void* scratch, size_t scratch_bytes,
                          hipStream_t st);
// LogUp multiplicities occ[t][i] (RawLookupTrace::get_trace's occurrence map)
hipError_t launch_lookup_occurrences(const Fr* comb, size_t n, uint32_t nt, const Fr* afil, const Fr* bfil,
                                     uint32_t* occ, void* scratch, size_t scratch_bytes, hipStream_t st);
// a_inverses / b_inverses / multiplicities columns from col_ainv on, and the LogUp terms
hipError_t launch_lookup_terms(const Fr* inv, const uint32_t* occ, const Fr* afil, size_t n, uint32_t nt, Fr* out,
                               size_t ostride, uint32_t col_ainv, Fr* term, hipStream_t st);

// ----------------------------------------------------- k_quotient.hip
struct QuotientArgs {
    const Fr* lde;      // N x w row-major, bit-reversed LDE
    uint32_t w;
    uint32_t logQ, log_q;
    const int32_t* air; // device copy of the AIR descriptor
    uint32_t air_len;
    Fr pub_alpha, pub_delta, alpha;
    Fr gen;             // coset shift GEN
    Fr wh_inv;          // w_h^-1 (last row point)
    const Fr* tabQ;     // two-level table of w_Q
    uint32_t L1;
    const Fr* zh;       // q values of Z_H on the coset (index i mod q)
    const Fr* inv_zh;   // their inverses
    const Fr* inv_den;  // 1/((x-1)(x-w_h^-1)) per computed point
    Fr* out;            // one value per computed point
    // Sharded evaluation: the points computed are i = i0 + (m << log_step),
    // m < n (n = 0: all Q points), and `lde` holds the LDE rows from global
    // row `row0` on.  Defaults: every point, the whole LDE.
    uint64_t i0 = 0;
    uint32_t log_step = 0;
    uint64_t row0 = 0;
    uint64_t n = 0;
    // the next-row LDE rows (point i + q), from global row `row0_next` on;
    // nullptr: in `lde` (every point's successor on the same rank)
    const Fr* lde_next = nullptr;
    uint64_t row0_next = 0;
    // thread order (launch_quotient sets it; LSP_QUOTIENT_ORDER): 1 = LDE row
    // order (a wave reads 64 adjacent rows, the default), 0 = point order
    uint32_t row_order = 0;
    // rows held at `lde` / `lde_next` (the debug build's bounds checks; 0 = not given)
    uint64_t lde_rows = 0, lde_next_rows = 0;
    // alpha-independent evaluation (prove.cpp, "constraints before alpha"): with
    // `cons` set, launch_quotient writes every constraint's value at each point
    // (ncons of them, in eval's order) as limb-planar 29-bit words, thread t's
    // value j limb l at cons[(j * 9 + l) * n + t], and folds nothing;
    // launch_quotient_fold then folds them with `alpha` and 1/Z_H into `out`
    uint32_t* cons = nullptr;
    uint32_t ncons = 0;
};
// den[m] = (x_i - 1)(x_i - w_h^-1), x_i = GEN * w_Q^i, i = i0 + (m << log_step), m < n
hipError_t launch_selector_denoms(const Fr* tabQ, uint32_t L1, Fr gen, Fr wh_inv, size_t n, Fr* den,
                                  hipStream_t st, uint64_t i0 = 0, uint32_t log_step = 0);
hipError_t launch_quotient(const QuotientArgs& a, hipStream_t st);
// out[m] = (sum_j alpha^(ncons-1-j) C_j) / Z_H from the values launch_quotient
// wrote into a.cons (same points, thread order and bounds as launch_quotient)
hipError_t launch_quotient_fold(const QuotientArgs& a, hipStream_t st);

// --------------------------------------------------------- k_open.hip
// den[i] = z - GEN * w_N^bitrev(row0 + i) for i < n (two-level table of w_N)
hipError_t launch_open_denoms(Fr z, Fr gen, const Fr* tabN, uint32_t L1, uint32_t logN, size_t n, Fr* den,
                              hipStream_t st, uint64_t row0 = 0);
// out[i] = c * inv_z[bitrev(bitrev(row0 + i) - step) - row0], i < n: the
// inverse denominators at z w_h from those at z (c = w_h^-1, step = N/h)
hipError_t launch_shift_inverse(const Fr* inv_z, Fr* out, Fr c, uint32_t logN, uint64_t step, uint64_t row0, size_t n,
                                hipStream_t st);
// partial sums for barycentric interpolation over rows [0, h):
// partial[b*w + c] = sum_{i in block b} M[i][c] * x_i * inv_den[i]
hipError_t launch_interp_partial(const Fr* M, uint32_t w, size_t h, const Fr* inv_den, Fr gen, const Fr* tabN,
                                 uint32_t L1, uint32_t logN, Fr* partial, uint32_t* nblocks, hipStream_t st,
                                 uint64_t row0 = 0);
// out[c] = sum_b partial[b*w + c]
hipError_t launch_sum_partials(const Fr* partial, uint32_t nblocks, uint32_t w, Fr* out, hipStream_t st);
struct ReduceArgs {
    const Fr* lde;  // N x w
    uint32_t w;
    const Fr* qlde; // N x q
    uint32_t q;
    const Fr* inv_z;   // 1/(zeta - x_i)
    const Fr* inv_zn;  // 1/(zeta_next - x_i)
    const Fr* apw;     // alpha_fri^k, k < 2w + q
    Fr ry_z, ry_zn;    // reduced opened values of the trace at zeta / zeta_next
    const Fr* ryq;     // opened value of each quotient chunk at zeta (q)
    Fr* out;           // N
    size_t n;
    F29* consts29 = nullptr;  // global scratch of reduce_rows_scratch(w, q) F29 (needed only beyond the LDS)
    size_t lds_max = 64 * 1024;  // the device's LDS per workgroup (lsp_ctx::lds_per_block)
};
// the reduce-rows constants stay in the workgroup's LDS up to the device's
// LDS per workgroup (lds_max: gfx950 160 KiB, i.e. w + 2q <= ~4,400 columns,
// read from the device at context creation); wider matrices keep them in
// global memory (ReduceArgs::consts29)
inline size_t reduce_rows_scratch(uint32_t w, uint32_t q, size_t lds_max) {
    const size_t lds = 3 * 64 * 16 + (w + 1 + 2 * (size_t)q) * 36;
    return lds <= lds_max ? 0 : w + 1 + 2 * (size_t)q;
}
hipError_t launch_reduce_rows(const ReduceArgs& a, hipStream_t st);
// one deliberately failing LSP_BOUNDS check (dbg_bounds.hpp; a no-op kernel in the product build)
hipError_t launch_bounds_probe(uint32_t* sink, hipStream_t st);
#ifdef LSP_DEBUG_BOUNDS
// each kernel translation unit's bounds-fault word ((file code << 16) | line, 0 = none), read and cleared
unsigned bounds_fault_k_ntt();
unsigned bounds_fault_k_hash();
unsigned bounds_fault_k_field();
unsigned bounds_fault_k_quotient();
unsigned bounds_fault_k_open();
unsigned bounds_fault_k_witness();
#endif
// one matrix opened at npts points (the generic reduce of TwoAdicFriPcs::open):
// ro[i] += sum_p (offys[p] - off[p] * sum_c apw[c] M[i][c]) * inv[p*n + i]
hipError_t launch_reduce_matrix(const Fr* M, size_t n, uint32_t w, const Fr* apw, uint32_t npts, const Fr* inv,
                                const Fr* off, const Fr* offys, Fr* ro, hipStream_t st);
// FRI fold of v (2m values) -> out (m values); tab: two-level table of w_{2M}^-1
// where M = 2^logm is the whole folded length (logm < 0: M = m) and v holds
// the pairs from global pair index i0 on (a shard of the vector).
hipError_t launch_fri_fold(const Fr* v, size_t m, Fr half, Fr half_beta, const Fr* tab, uint32_t L1,
                           Fr* out, hipStream_t st, uint64_t i0 = 0, int logm = -1);

}  // namespace lsp
