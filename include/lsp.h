/*
 * lsp.h -- C-ABI of liblsp_hip.so, the MI355X-native hot path of
 * distributed-lab/linea-stark-prover.
 *
 * The reference plugs its prover together from Plonky3 type aliases
 * (bin/src/config.rs:9-25) and calls p3_uni_stark::prove/verify
 * (bin/src/main.rs:80-96).  Every entry point below replaces one trait method
 * or free function reachable from that plug point; the comment on each cites
 * the reference call site (file:line in the reference repo) and the Plonky3
 * item ([EXT] = distributed-lab/Plonky3@f888f90, Cargo.lock:505-711, not
 * vendored) it stands in for.  INTEGRATION.md shows the Rust-side binding.
 *
 * Conventions
 *   - Elements: lsp_fr = 4 x u64 little-endian limbs in Montgomery form with
 *     R = 2^256, canonical in [0, r) -- ark-ff 0.5's in-memory Fr, so a
 *     &[Bls12_377Fr] can be passed as *const lsp_fr once the shim asserts
 *     size_of::<Bls12_377Fr>() == 32.
 *   - Matrices: row-major, height x width (p3-matrix RowMajorMatrix).
 *   - `mem`: LSP_MEM_HOST = pointers are host memory (copied in/out),
 *     LSP_MEM_DEVICE = pointers are device memory on the context's GPU
 *     (allocated with lsp_dev_alloc or any HIP allocation on that device).
 *   - Errors: every call returns LSP_OK (0) or an LSP_E_* code; the message is
 *     in lsp_last_error(ctx).  Plonky3 panics where these return non-zero, so
 *     the Rust shim panics on non-zero status (except verify).
 *   - Threading: a context is bound to one device and one HIP stream and is
 *     serialised by an internal mutex; calls are synchronous at return.
 */
#ifndef LSP_H
#define LSP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { uint64_t l[4]; } lsp_fr;

enum {
    LSP_OK = 0,
    LSP_E_ARG = 1,     /* bad argument (null pointer, bad descriptor, ...) */
    LSP_E_OOM = 2,     /* device or host allocation failed */
    LSP_E_HIP = 3,     /* HIP runtime error */
    LSP_E_SIZE = 4,    /* height not a power of two / too large */
    LSP_E_VERIFY = 5,  /* proof rejected */
    LSP_E_STATE = 6    /* no GPU / context unusable */
};

enum { LSP_MEM_HOST = 0, LSP_MEM_DEVICE = 1 };

/* AIR descriptor (int32 array) -- the AirConfig list of LineaAIR
 * (air/src/lib.rs:11-54), i.e. what LineaAIR::eval iterates:
 *   [n_configs, config_0, config_1, ...]
 * LSP_AIR_PERMUTATION (AirPermutationConfig, air/src/air_permutation.rs:1-24):
 *   1, na, nb, a_ids[na], b_ids[nb], b_inverse_id, check_id
 * LSP_AIR_LOOKUP (AirLookupConfig, air/src/air_lookup.rs:1-40):
 *   2, na, a_ids[na], ntables, ncols, b_ids[ntables*ncols], a_filter_id,
 *   b_filter_ids[ntables], a_inverses_id, b_inverses_ids[ntables],
 *   occurrences_ids[ntables], check_id
 * Column ids are absolute (already shifted, trace/src/lib.rs:40-58). */
enum { LSP_AIR_PERMUTATION = 1, LSP_AIR_LOOKUP = 2 };

typedef struct lsp_ctx lsp_ctx;
typedef struct lsp_tree lsp_tree;
typedef struct lsp_proof lsp_proof;

/* StarkConfig / FriConfig / Perm parameters (bin/src/config.rs:9-25,
 * bin/src/main.rs:49-64).
 * struct_size must be sizeof(lsp_params) as the caller compiled it (88
 * bytes on LP64 for this layout): lsp_ctx_create rejects any other
 * value with LSP_E_ARG, so a caller built against an older layout (whose
 * first field was sbox_degree = 11 or 17) fails loudly instead of having
 * its stack read as the newer fields. */
typedef struct {
    uint32_t struct_size;          /* sizeof(lsp_params) */
    uint32_t sbox_degree;          /* U1: 11 (default) or 17 */
    uint32_t rounds_f;             /* full rounds, 8 (bin/src/main.rs:49) */
    uint32_t rounds_p;             /* partial rounds, 22 (bin/src/main.rs:49) */
    const lsp_fr *round_constants; /* 3*rounds_f + rounds_p, new_from_rng order:
                                      initial external, terminal external, internal */
    uint32_t log_blowup;           /* 3  (bin/src/main.rs:59) */
    uint32_t log_final_poly_len;   /* 0  (bin/src/main.rs:60) */
    uint32_t num_queries;          /* 33 (bin/src/main.rs:61) */
    uint32_t proof_of_work_bits;   /* 0  (bin/src/main.rs:62) */
    int32_t public_degree;         /* U6: symbolic degree of a public value, 1 (fork, default) or 0 */
    /* U2/U3: the linear layers of Poseidon2Bls12337<3> (the fork's
     * Poseidon2InternalLayer / Poseidon2ExternalLayer for WIDTH = 3, [EXT
     * p3-bls12-377-fr]); NULL = the default, which is upstream Plonky3's
     * width-3 template (p3-bn254-fr):
     *   internal_diag  3 elements d: s_i <- (s0 + s1 + s2) + d_i s_i, i.e.
     *                  M_I = J + diag(d); default d = (1, 1, 2)
     *   external_mds   9 elements, row-major M_E: s <- M_E s before the first
     *                  full round and after every full round; default
     *                  circ(2, 1, 1), i.e. s_i += s0 + s1 + s2
     * Montgomery form like round_constants.  Non-default layers cost 12
     * products per full round and 3 per partial round more than the default
     * (additions only) on every path: device, host scalar and host IFMA. */
    const lsp_fr *internal_diag;
    const lsp_fr *external_mds;
    /* Transcript conventions of the fork's p3-uni-stark / p3-fri /
     * HashChallenger ([EXT], bin/src/config.rs:23, bin/src/main.rs:78,88-96),
     * which no reference artefact pins.  0 = the
     * default for every field, so a zero-filled tail keeps today's proofs.
     *   U7  skip_log_degree        1: log2(h) is not observed before the trace root
     *       skip_public_values     1: the public values [alpha, delta] are not
     *                              observed before the quotient challenge
     *       observe_opened_values  1: TwoAdicFriPcs::open observes every opened
     *                              value (trace at zeta, trace at zeta*w_h,
     *                              chunk j at zeta, in that order) before it
     *                              samples alpha_fri (later upstream Plonky3)
     *   U8  sample_bits_montgomery 1: sample_bits (query indices and the PoW
     *                              check) takes the low bits of the Montgomery
     *                              form instead of the canonical value
     *   U12 skip_final_poly        1: the final polynomial's coefficients are
     *                              not observed before grinding
     * The switches are not recorded in the proof (the wire format, DESIGN.md
     * §9, and p3_uni_stark::Proof<SC> have no field for them): prover and
     * verifier must be configured alike.  A proof made under other conventions
     * fails lsp_verify (and the reference's verify) with LSP_E_VERIFY at the
     * first challenge-dependent check -- an opened value's Merkle path or the
     * quotient identity at zeta -- and nothing in the bytes names the cause. */
    uint32_t skip_log_degree;
    uint32_t skip_public_values;
    uint32_t observe_opened_values;
    uint32_t sample_bits_montgomery;
    uint32_t skip_final_poly;
} lsp_params;

/* ---------------------------------------------------------------- library */
/* "... (gfx950)", or "... (gfx950, debug-bounds)" for the bounds-checked
 * debug build (python -m linea_stark_prover_amd.build --debug-bounds ->
 * liblsp_hip_dbg.so): every kernel checks its geometry-derived
 * indices, a failed check skips the access (no fault) and fails the C-ABI
 * call that launched it with LSP_E_STATE "device bounds check failed at
 * <file>:<line>". */
const char *lsp_version(void);
/* the debug build's self-test: one deliberately failing check on the device,
 * so LSP_E_STATE with that message; the product build answers LSP_E_STATE
 * "not a debug-bounds build" */
int lsp_debug_bounds_probe(lsp_ctx *ctx);
int lsp_device_count(int *n);
const char *lsp_last_error(const lsp_ctx *ctx);

/* U4/U5: documented seeded generator replacing thread_rng() for the
 * challenges (bin/src/main.rs:29-31) and Perm::new_from_rng (bin/src/main.rs:49).
 * round_constants must hold 3*rounds_f + rounds_p elements. */
int lsp_seeded_setup(uint64_t seed, uint32_t rounds_f, uint32_t rounds_p, lsp_fr *alpha, lsp_fr *delta,
                     lsp_fr *round_constants);

/* Field conversions (host).  from_be_bytes_mod_order replaces
 * FF_Bls12_377Fr::from_be_bytes_mod_order (trace/src/permutation.rs:102-104).
 * These helpers (and lsp_fri_fold_row) return nothing; a NULL argument makes
 * them a no-op.  Every int-returning entry point reports NULL arguments as
 * LSP_E_ARG (tests/test_abi_sweep.py). */
void lsp_fr_from_canonical(const uint64_t in[4], lsp_fr *out);
void lsp_fr_to_canonical(const lsp_fr *in, uint64_t out[4]);
void lsp_fr_from_be_bytes_mod_order(const uint8_t *be, size_t n, lsp_fr *out);
void lsp_fr_mul(const lsp_fr *a, const lsp_fr *b, lsp_fr *out);
void lsp_fr_inv(const lsp_fr *a, lsp_fr *out);
void lsp_two_adic_generator(uint32_t bits, lsp_fr *out); /* TwoAdicField::two_adic_generator */

/* ---------------------------------------------------------------- context */
/* device = LSP_HOST_ONLY creates a verifier-only context that never touches
 * a GPU (lsp_verify, lsp_merkle_verify work; device entry points return
 * LSP_E_STATE). */
#define LSP_HOST_ONLY (-1)
int lsp_ctx_create(int device, const lsp_params *params, lsp_ctx **out);
int lsp_ctx_destroy(lsp_ctx *ctx);
int lsp_synchronize(lsp_ctx *ctx);
int lsp_dev_alloc(lsp_ctx *ctx, size_t bytes, void **dptr);
int lsp_dev_free(lsp_ctx *ctx, void *dptr);
int lsp_memcpy_h2d(lsp_ctx *ctx, void *dst, const void *src, size_t bytes);
int lsp_memcpy_d2h(lsp_ctx *ctx, void *dst, const void *src, size_t bytes);

/* ------------------------------------------------------------------- Dft */
/* TwoAdicSubgroupDft::coset_lde_batch(mat, added_bits, shift) followed by
 * .bit_reverse_rows().to_row_major_matrix(), as TwoAdicFriPcs::commit uses it
 * ([EXT p3-dft Radix2DitParallel], bin/src/config.rs:22; bin/src/main.rs:52).
 * in: h x w values on H_h; out: (h << added_bits) x w, row i = p(shift * w_N^bitrev(i)). */
int lsp_coset_lde_batch(lsp_ctx *ctx, const lsp_fr *in, size_t h, size_t w, uint32_t added_bits,
                        const lsp_fr *shift, lsp_fr *out, int mem);
/* Same with one shift per column (the quotient-chunk commit of p3-uni-stark,
 * where chunk j uses GEN / (GEN * w_Q^j)). */
int lsp_coset_lde_batch_shifts(lsp_ctx *ctx, const lsp_fr *in, size_t h, size_t w, uint32_t added_bits,
                               const lsp_fr *shifts, lsp_fr *out, int mem);
/* The rest of the TwoAdicSubgroupDft surface ([EXT p3-dft]; Radix2DitParallel
 * is the reference's Dft, bin/src/config.rs:22), h = 2^k >= 1, w >= 1:
 * coset_dft_batch(mat, shift) (dft_batch: shift = NULL, i.e. 1):
 *   coeffs: h x w true coefficients, row i = c_i; out: h x w evaluations on
 *   shift * H_h stored bit-reversed, row j = p(shift * w_h^bitrev(j)) -- the
 *   Evaluations = BitReversedMatrixView layout Radix2DitParallel returns.
 * coset_idft_batch(mat, shift) (idft_batch: shift = NULL):
 *   evals: h x w natural order, row i = p(shift * w_h^i); out: h x w
 *   coefficients, canonical.  shift must be nonzero.
 * lde_batch(mat, added_bits) is lsp_coset_lde_batch with shift 1. */
int lsp_coset_dft_batch(lsp_ctx *ctx, const lsp_fr *coeffs, size_t h, size_t w, const lsp_fr *shift, lsp_fr *out,
                        int mem);
int lsp_coset_idft_batch(lsp_ctx *ctx, const lsp_fr *evals, size_t h, size_t w, const lsp_fr *shift, lsp_fr *out,
                         int mem);

/* ---------------------------------------------------- Poseidon2 / symmetric */
/* Poseidon2Bls12337<3>::permute_mut on n states of 3 (bin/src/config.rs:11) */
int lsp_poseidon2_permute_batch(lsp_ctx *ctx, lsp_fr *states, size_t n, int mem);
/* PaddingFreeSponge<Perm,3,2,1>::hash_iter of each of n rows of width w
 * (bin/src/config.rs:12) */
int lsp_hash_rows(lsp_ctx *ctx, const lsp_fr *rows, size_t n, size_t w, lsp_fr *out, int mem);

/* ------------------------------------------------------------------ Mmcs */
/* MerkleTreeMmcs::commit over nmats equal-height row-major matrices
 * (bin/src/config.rs:19-20): leaf = hash_iter of the rows concatenated in
 * commit order (U11); nodes = CompressionFunctionFromHasher (bin/src/config.rs:17). */
int lsp_merkle_commit(lsp_ctx *ctx, const lsp_fr *const *mats, const size_t *widths, size_t nmats,
                      size_t height, int mem, lsp_fr *root, lsp_tree **tree);
/* Mmcs::open_batch: rows_out gets sum(widths) elements, path_out log2(height) digests */
int lsp_merkle_open(const lsp_tree *tree, size_t index, lsp_fr *rows_out, lsp_fr *path_out);
/* digest layer `level` (0 = leaf digests) -> out (height >> level elements) */
int lsp_merkle_layer(const lsp_tree *tree, uint32_t level, lsp_fr *out);
/* Mmcs::verify_batch (host) -- LSP_OK or LSP_E_VERIFY */
int lsp_merkle_verify(const lsp_ctx *ctx, const lsp_fr *root, const size_t *widths, size_t nmats,
                      uint32_t log_height, size_t index, const lsp_fr *rows, const lsp_fr *path);
int lsp_tree_free(lsp_tree *tree);

/* ----------------------------------------------------------- FriFolder */
/* TwoAdicFriGenericConfig::fold_matrix(beta, RowMajorMatrix(v, 2)) [EXT p3-fri]:
 * out[i] = (1/2 + beta/2 g^-bitrev(i)) v[2i] + (1/2 - beta/2 g^-bitrev(i)) v[2i+1],
 * g = w_len.  len = length of v (power of two >= 2); out has len/2. */
int lsp_fri_fold(lsp_ctx *ctx, const lsp_fr *v, size_t len, const lsp_fr *beta, lsp_fr *out, int mem);
/* TwoAdicFriGenericConfig::fold_row (host; verifier side) */
void lsp_fri_fold_row(size_t index, uint32_t log_height, const lsp_fr *beta, const lsp_fr *e0,
                      const lsp_fr *e1, lsp_fr *out);

/* ------------------------------------------------------------- quotient */
/* log_quotient_degree from the symbolic constraint degrees (U6 rule) */
int lsp_log_quotient_degree(const int32_t *air, size_t air_len, int32_t public_degree, uint32_t *log_q);
/* p3-uni-stark quotient_values over the LDE of the trace (row-major,
 * bit-reversed, (h << log_blowup) x w) with LineaAIR::eval
 * (air/src/lib.rs:47-167): out[i], i < h << log_q, natural order on GEN*H_Q. */
int lsp_quotient_values(lsp_ctx *ctx, const lsp_fr *lde, size_t h, size_t w, const int32_t *air, size_t air_len,
                        const lsp_fr *public_values, size_t npub, const lsp_fr *alpha, lsp_fr *out, int mem);

/* ------------------------------------------------------------- PCS open */
/* interpolate_coset [EXT p3-interpolation] of the first h rows of a bit-reversed
 * LDE (the low coset shift*H_h) at z: ys_out gets w values (host memory). */
int lsp_interpolate_coset(lsp_ctx *ctx, const lsp_fr *lde_bitrev, size_t h, size_t w, const lsp_fr *shift,
                          const lsp_fr *z, lsp_fr *ys_out, int mem);
/* compute_inverse_denominators of TwoAdicFriPcs::open [EXT p3-fri], reached
 * from p3_uni_stark::prove (bin/src/main.rs:80-86) through pcs.open:
 * out[p*N + i] = 1 / (points[p] - shift * w_N^bitrev(i)), N = 2^log_n, i.e.
 * against the bit-reversed LDE domain shift*H_N (shift = GENERATOR there).
 * Every point must lie outside that coset.  out: npoints * N elements. */
int lsp_inverse_denominators(lsp_ctx *ctx, const lsp_fr *points, size_t npoints, uint32_t log_n,
                             const lsp_fr *shift, lsp_fr *out, int mem);
/* The "reduce rows" step of TwoAdicFriPcs::open [EXT p3-fri] for one matrix
 * (n rows of width w, bit-reversed LDE) opened at npoints points:
 *   for each point p: ro[i] += off * (sum_c alpha^c ys[p][c] - sum_c alpha^c M[i][c]) * inv_denoms[p*n + i];
 *                     off *= alpha^w
 * ys: npoints x w (host memory); alpha_pow_offset (host, in/out) is the running
 * alpha^{num_reduced} of this log-height, advanced as Plonky3 advances it, so
 * successive calls over the opened matrices in commit order build the FRI
 * input vector ro (n elements, in/out). */
int lsp_open_reduce(lsp_ctx *ctx, const lsp_fr *mat, size_t n, size_t w, const lsp_fr *inv_denoms, const lsp_fr *ys,
                    size_t npoints, const lsp_fr *alpha, lsp_fr *alpha_pow_offset, lsp_fr *ro, int mem);
/* The host side of MerkleTreeMmcs::commit (the tree tops below
 * host_tree_top digests): CompressionFunctionFromHasher on n pairs
 * (pairs[2i], pairs[2i+1]) -> out[i], and PaddingFreeSponge::hash_iter of n
 * rows of width w -> out[i], on the CPU (8 at a time with AVX-512 IFMA when the
 * CPU has it, else 4 x 64-bit scalar).  Host memory; works on a host-only
 * context. */
int lsp_host_compress_batch(const lsp_ctx *ctx, const lsp_fr *pairs, size_t n, lsp_fr *out);
int lsp_host_hash_rows(const lsp_ctx *ctx, const lsp_fr *rows, size_t n, size_t w, lsp_fr *out);
/* p3-field batch_multiplicative_inverse */
int lsp_batch_inverse(lsp_ctx *ctx, const lsp_fr *in, size_t n, lsp_fr *out, int mem);

/* ----------------------------------------------------------------- prove */
/* p3_uni_stark::prove(config, air, challenger, trace, public_values)
 * (bin/src/main.rs:80-86) with Challenger = HashChallenger::new(vec![], hash)
 * (bin/src/main.rs:78).  trace: h x w row-major. */
int lsp_prove(lsp_ctx *ctx, const lsp_fr *trace, size_t h, size_t w, const int32_t *air, size_t air_len,
              const lsp_fr *public_values, size_t npub, int mem, lsp_proof **out);
/* Sharded prove: one proof over G = 2^b ranks,
 * G <= 2^(log_blowup + 6) and at least 2 LDE rows per rank (LSP_E_ARG /
 * LSP_E_SIZE otherwise).  Rank g owns the LDE rows [g N/G, (g+1) N/G) --
 * whole cosets of the bit-reversed LDE while G <= 2^log_blowup, a sub-coset
 * of N/G < h rows beyond, in either case a whole
 * subtree of each input Merkle tree -- the quotient points whose rows it
 * holds and a slice of every FRI vector; ranks exchange subtree roots, the
 * trace coefficients, the quotient chunks, the opened values, short FRI
 * vectors and the query openings.  The proof is byte-identical to
 * lsp_prove's.
 * In-process group: rank g = ctxs[g]; distinct devices (one host process
 * driving the node's GPUs, exchanges device-to-device with peer access) or
 * the same device repeated (virtual ranks).  traces[g] is rank g's copy of
 * the trace (mem as in lsp_prove; device pointers on ctxs[g]'s device).
 * Replaces p3_uni_stark::prove (bin/src/main.rs:80-86) like lsp_prove. */
typedef struct lsp_group lsp_group;
int lsp_group_create(lsp_ctx *const *ctxs, int n, lsp_group **out);
int lsp_group_destroy(lsp_group *grp);
int lsp_prove_group(lsp_group *grp, const lsp_fr *const *traces, size_t h, size_t w, const int32_t *air,
                    size_t air_len, const lsp_fr *public_values, size_t npub, int mem, lsp_proof **out);
/* Process-per-GPU sharding: each of the G processes attaches a communicator
 * to its context (rank g of G), then all call lsp_prove_sharded together;
 * ranks, data layout and result are those of lsp_prove_group.
 *   lsp_comm_ops   the caller's transport over host buffers (allgather: recv
 *                  receives size * bytes in rank order; bcast: root's buf to
 *                  every rank); callbacks return 0 on success.
 *   RCCL           device-direct over xGMI: rank 0 creates the id with
 *                  lsp_comm_rccl_unique_id, the caller distributes its 128
 *                  bytes, every rank calls lsp_ctx_attach_rccl (collective). */
typedef struct lsp_comm_ops {
    int rank, size;
    void *user;
    int (*allgather)(void *user, const void *send, void *recv, size_t bytes);
    int (*bcast)(void *user, void *buf, size_t bytes, int root);
} lsp_comm_ops;
int lsp_ctx_attach_comm_ops(lsp_ctx *ctx, const lsp_comm_ops *ops);
int lsp_comm_rccl_unique_id(uint8_t id[128]);
int lsp_ctx_attach_rccl(lsp_ctx *ctx, const uint8_t id[128], int rank, int size);
int lsp_ctx_detach_comm(lsp_ctx *ctx);
/* Rehearsal transport: this context plays rank `rank` of a `size`-rank
 * lsp_prove_sharded on its one GPU, every peer's part of an exchange
 * fabricated locally (allgather slots of other ranks = a copy of this rank's
 * payload, broadcasts from other roots = zeros).  The proof is NOT valid and
 * is marked so: lsp_proof_serialize answers only the size query (buf = NULL)
 * and lsp_proof_get_view refuses it (LSP_E_STATE).  The call measures one
 * rank's device memory, phase times and collective schedule (lsp_comm_log) at
 * full size (e.g.
 * BASELINE configs[3], 2^26 rows over 8 GPUs, one rank at a time on one GPU;
 * tools/rank_rehearsal.py). */
int lsp_ctx_attach_loopback(lsp_ctx *ctx, int rank, int size);
/* device memory of the context: pool_bytes = its grow-only buffer pool (the
 * high-water mark of its working set), device_used / device_total =
 * hipMemGetInfo of its GPU */
int lsp_ctx_mem_stats(lsp_ctx *ctx, size_t *pool_bytes, size_t *device_used, size_t *device_total);
/* collective check of the attached communicator: an allgather and a
 * broadcast of known patterns (LSP_E_STATE on wrong data).  With more than one
 * rank it then calibrates the exchange: the allgather bandwidth into one rank
 * (a 4 MiB probe, then 256 MiB unless the first is below 20 GB/s) and this
 * GPU's inverse-NTT rate, the minimum of each over the ranks.  The sharded
 * proofs choose their inverse-NTT exchange on those numbers (SURVEY 8(e) step
 * 1: split by columns + an allgather of the coefficients, or a redundant
 * inverse on every rank; lsp_comm_exchange_plan) */
int lsp_comm_selftest(lsp_ctx *ctx);
/* the exchange plan a sharded proof of an h x w trace with q quotient chunks
 * (lsp_log_quotient_degree; 0 = count the trace only) makes on ctx's
 * communicator: the calibrated allgather_gbs / intt_gelem_s (0 when the
 * communicator was never self-tested), the probe's size, split (1 = columns
 * split + allgather, 0 = redundant inverse on every rank) and the model's two
 * costs in ms.  Any output but split may be NULL.  LSP_SHARD_SPLIT_INTT=0/1
 * in the environment forces the choice. */
int lsp_comm_exchange_plan(lsp_ctx *ctx, size_t h, size_t w, size_t q, double *allgather_gbs, double *intt_gelem_s,
                           size_t *probe_bytes, int *split, double *allgather_ms, double *redundant_ms);
/* every rank's own calibration probes, rank order, 3 doubles per rank:
 * allgather GB/s of the 4 MiB probe, of the 256 MiB probe (0: not run, the
 * small one was below 20 GB/s on some rank), inverse-NTT G elements/s on
 * random data -- the raw values whose minimum lsp_comm_exchange_plan uses.
 * *n = 3 x ranks (0 when never calibrated); out == NULL or cap < *n -> only *n */
int lsp_comm_calibration(lsp_ctx *ctx, double *per_rank, size_t cap, size_t *n);
/* the quotient-chunk broadcasts a sharded proof of h rows with q chunks
 * issues on ctx's communicator (either inverse-NTT exchange): how many, the
 * bytes of each, and their total time at the calibrated allgather bandwidth
 * (0 when uncalibrated); at 2^26 rows over 8 ranks: 4 x 2 GiB.  Any output
 * may be NULL. */
int lsp_comm_quotient_exchange(lsp_ctx *ctx, size_t h, size_t q, size_t *bcasts, size_t *bytes_each,
                               double *model_ms);
/* threads of ctx's host pool (tree tops, FRI tail, query assembly): up to 16,
 * from this process's CPU affinity set divided among LOCAL_WORLD_SIZE ranks
 * (the library cannot tell a set the ranks share from a slice pinned for this
 * rank alone, and divides).  LSP_HOST_THREADS overrides: a launcher that pins
 * each rank to CPUs of its own sets it (the Python launch path,
 * replicas.init_from_env, compares the ranks' sets and sets it exactly) */
int lsp_ctx_host_threads(lsp_ctx *ctx, int *n);
/* rank and size of the attached communicator (LSP_E_STATE if none) */
int lsp_comm_info(lsp_ctx *ctx, int *rank, int *size);
/* The collective schedule of the last lsp_prove_sharded on ctx, one entry
 * per collective in issue order: ops[i] 'A' (allgather; bytes[i] = each
 * rank's share) or 'B' (broadcast; bytes[i] = the buffer, roots[i] = its
 * root; -1 for allgathers), tags[i] what it carried ("trace coefficients",
 * "quotient chunk coefficients", "trace subtree roots", "FRI vector", ...;
 * strings live until the next prove on ctx), ms[i] the device time between
 * events recorded around it on ctx's stream (the wait for the slowest peer
 * included).  init_ms = the communicator's creation time (RCCL:
 * ncclCommInitRank; 0 for the other transports).  Any output array may be
 * NULL; *n = the number of entries (at most cap are written).  Every rank of
 * a proof must log the same (op, bytes, root) sequence: RCCL hangs otherwise
 * (tests/test_gpu_configs_full.py checks it at BASELINE configs[3]'s size). */
int lsp_comm_log(lsp_ctx *ctx, char *ops, size_t *bytes, int *roots, double *ms, const char **tags, size_t cap,
                 size_t *n, double *init_ms);
int lsp_prove_sharded(lsp_ctx *ctx, const lsp_fr *trace, size_t h, size_t w, const int32_t *air, size_t air_len,
                      const lsp_fr *public_values, size_t npub, int mem, lsp_proof **out);
/* serialized proof (format in DESIGN.md); buf == NULL -> *len = required size */
int lsp_proof_serialize(const lsp_proof *proof, uint8_t *buf, size_t cap, size_t *len);
/* the inverse (untrusted bytes: LSP_E_ARG on anything malformed) */
int lsp_proof_deserialize(const uint8_t *buf, size_t len, lsp_proof **out);
int lsp_proof_free(lsp_proof *proof);

/* ------------------------------------------------------------- Proof<SC> */
/* Field-by-field view of a proof, one field per field of
 * p3_uni_stark::Proof<SC> ([EXT p3-uni-stark proof.rs]; built at
 * bin/src/main.rs:80-86, read by p3_uni_stark::verify at bin/src/main.rs:88-96)
 * for the reference's Config (bin/src/config.rs:19-25: Val = Challenge = Fr,
 * MerkleTreeMmcs<Val,Val,Hash,Compress,1>, TwoAdicFriPcs):
 *   degree_bits                         <- degree_bits
 *   commitments.trace                   <- Hash::from([*trace_commit])
 *   commitments.quotient_chunks         <- Hash::from([*quotient_commit])
 *   opened_values.trace_local / _next   <- trace_local[width] / trace_next[width]
 *   opened_values.quotient_chunks[j]    <- vec![quotient_chunks[j]]   (j < 2^log_quotient_chunks)
 *   opening_proof: FriProof {
 *     commit_phase_commits[r]           <- Hash::from([fri_commits[r]])
 *     final_poly                        <- final_poly[final_poly_len]
 *     pow_witness                       <- *pow_witness
 *     query_proofs[i]: QueryProof {
 *       input_proof: vec![               (one BatchOpening per committed round)
 *         BatchOpening { opened_values: vec![trace_rows[i]],
 *                        opening_proof: trace_paths[i] as Vec<[Fr; 1]> },
 *         BatchOpening { opened_values: (0..q).map(|j| vec![quotient_rows[i][j]]),
 *                        opening_proof: quotient_paths[i] as Vec<[Fr; 1]> } ],
 *       commit_phase_openings[r]: CommitPhaseProofStep {
 *         sibling_value: fri_siblings[i][r],
 *         opening_proof: fri_paths[i][r] (fri_path_lens[r] digests) } } }
 * Arrays are query-major (query i's trace row at trace_rows + i*width, its
 * round-r FRI path after the paths of rounds < r); paths list siblings leaf
 * to root.  Elements are lsp_fr (Montgomery, canonical).  The pointers stay
 * valid until lsp_proof_free.  rust/p3-hip/src/proof.rs builds Proof<SC>
 * from this view and back. */
typedef struct {
    uint32_t degree_bits;          /* log2 of the trace height */
    uint32_t log_quotient_chunks;  /* q = 2^log_quotient_chunks */
    uint32_t width;                /* trace width w */
    uint32_t num_queries;
    uint32_t num_fri_rounds;
    uint32_t final_poly_len;
    uint32_t input_path_len;       /* Merkle path length of the trace and quotient openings */
    const uint32_t *fri_path_lens; /* [num_fri_rounds] */
    const lsp_fr *trace_commit, *quotient_commit, *pow_witness;
    const lsp_fr *trace_local, *trace_next, *quotient_chunks;
    const lsp_fr *fri_commits, *final_poly;
    const lsp_fr *trace_rows, *trace_paths;        /* num_queries x width, num_queries x input_path_len */
    const lsp_fr *quotient_rows, *quotient_paths;  /* num_queries x q, num_queries x input_path_len */
    const lsp_fr *fri_siblings, *fri_paths;        /* num_queries x rounds, num_queries x sum(fri_path_lens) */
} lsp_proof_view;
int lsp_proof_get_view(const lsp_proof *proof, lsp_proof_view *view);
/* a proof handle from a view (copies; e.g. a Proof<SC> made elsewhere, for
 * lsp_proof_serialize / lsp_verify); LSP_E_ARG on null or non-canonical data */
int lsp_proof_from_view(const lsp_proof_view *view, lsp_proof **out);
/* p3_uni_stark::verify (bin/src/main.rs:88-96) on the host CPU */
int lsp_verify(const lsp_ctx *ctx, const int32_t *air, size_t air_len, const lsp_fr *public_values, size_t npub,
               const uint8_t *proof, size_t len);
/* per-phase device times of the last lsp_prove (ms), span names as in the
 * reference's bench.log */
int lsp_last_timings(const lsp_ctx *ctx, double *ms, const char **names, size_t cap, size_t *n);
/* Which phases the following proofs time (two device events each, ~0.3 ms
 * of host API time per 2^19 proof for all of them): on = 0 none, on != 0
 * with n_only = 0 all (the default), else only the phases named in only[]
 * (span names as lsp_last_timings reports them).  lsp_last_timings reports
 * the phases timed.  Proof bytes are the same either way. */
int lsp_ctx_set_phase_timing(lsp_ctx *ctx, int on, const char *const *only, size_t n_only);
/* the last lsp_prove's data-shaped operations in order, worded as the
 * reference's tracing spans with dims (bench.log:19-64), e.g.
 * "coset_lde_batch dims: 14x524288 | added_bits: 3",
 * "reduce matrix quotient dims: 1x4194304", "divide_by_height dims: 1x8";
 * strings live until the next prove on ctx */
int lsp_last_spans(const lsp_ctx *ctx, const char **lines, size_t cap, size_t *n);

/* Witness generation on the device: the trace crate's
 * RawPermutationTrace::get_trace (trace/src/permutation.rs:24-93) and
 * RawLookupTrace::get_trace (trace/src/lookup.rs:46-176).  Raw columns are
 * column-major (column k at ptr + k*n; lookup B: table t column c at
 * (t*nbc + c)*n; b_filter: table t at t*n); the block's columns are written
 * into rows of a row-major trace of width trace_w from column col0 on -- the
 * layout RawTrace::get_trace assembles (trace/src/lib.rs:94-106), so the
 * blocks of one trace are generated in push order into one buffer.
 *   permutation block: a.., b.., b_inverse, check             (na + nb + 2)
 *   lookup block: a.., b.., a_filter, b_filters.., a_inverses, b_inverses..,
 *                 multiplicities.., prefix sum                (na + nt(nbc+3) + 3)
 * LSP_E_STATE if the check column does not end at 1 (permutation) / 0
 * (lookup), as the reference asserts.  mem applies to every pointer. */
int lsp_witness_permutation(lsp_ctx *ctx, const lsp_fr *a, uint32_t na, const lsp_fr *b, uint32_t nb, size_t n,
                            const lsp_fr *alpha, const lsp_fr *delta, lsp_fr *trace, size_t trace_w, size_t col0,
                            int mem);
int lsp_witness_lookup(lsp_ctx *ctx, const lsp_fr *a, uint32_t na, const lsp_fr *b, uint32_t ntables, uint32_t nbc,
                       const lsp_fr *a_filter, const lsp_fr *b_filter, size_t n, const lsp_fr *alpha,
                       const lsp_fr *delta, lsp_fr *trace, size_t trace_w, size_t col0, int mem);

/* Trace input: one CBOR RawPermutationTrace
 * (trace/src/permutation.rs:9-22) or RawLookupTrace (trace/src/lookup.rs:
 * 10-44) as serde/ciborium write them ([u8; 32] words big-endian, reduced
 * with from_be_bytes_mod_order; missing lookup filter entries = 1, as
 * read_file pads them).  kind = LSP_AIR_PERMUTATION / LSP_AIR_LOOKUP;
 * permutation: ntables = number of b columns, nbc = 0.
 * lsp_raw_trace_push = RawTrace::push_permutation / push_lookup
 * (trace/src/lib.rs:38-60): resize to `height` (zero words) and generate the
 * block's witness on the GPU into trace columns col0 .. col0 + width - 1. */
typedef struct lsp_raw_trace lsp_raw_trace;
int lsp_raw_trace_parse(const uint8_t *cbor, size_t len, lsp_raw_trace **out);
int lsp_raw_trace_shape(const lsp_raw_trace *t, int *kind, uint32_t *na, uint32_t *ntables, uint32_t *nbc,
                        size_t *max_height, size_t *width);
/* raw columns resized to `height`, column-major (a.., b.. table-major,
 * lookup: a_filter, b_filters..); out == NULL -> *n = element count */
int lsp_raw_trace_columns(const lsp_raw_trace *t, size_t height, lsp_fr *out, size_t cap, size_t *n);
int lsp_raw_trace_push(lsp_ctx *ctx, const lsp_raw_trace *t, size_t height, const lsp_fr *alpha, const lsp_fr *delta,
                       lsp_fr *trace, size_t trace_w, size_t col0, int mem);
int lsp_raw_trace_free(lsp_raw_trace *t);

/* Fr-multiplication throughput of the device multiplier (register-resident
 * independent chains): the calibrated VALU peak the Merkle/Poseidon2
 * roofline is quoted against. */
int lsp_calibrate_fr_mul(lsp_ctx *ctx, double *gmul_per_s);
/* Poseidon2-w3 permutation throughput (register-resident chained states,
 * the device permutation kernels' code): the peak the Merkle kernels'
 * roofline (bench.py roofline_valu) is quoted against, in M perm/s. */
int lsp_calibrate_poseidon2(lsp_ctx *ctx, double *mperm_per_s);
/* this GPU's inverse-NTT rate in G elements/s on an h x w matrix of seeded
 * random field elements (h = 2^log_h): the median of 5 timed inverse NTTs
 * after a warm-up, the probe lsp_comm_selftest calibrates the exchange with
 * (log_h 20, w 8) -- random operands, not zeros, since this chip is
 * power-held on MAD-dense work.  At most 2^28 elements (LSP_E_ARG beyond) */
int lsp_calibrate_intt(lsp_ctx *ctx, uint32_t log_h, size_t w, double *gelem_per_s);

/* ------------------------------------------------------------- witness */
/* Synthetic permutation trace with the witness columns of
 * RawPermutationTrace::get_trace (trace/src/permutation.rs:24-93):
 * row-major h x (2*ncols + 2), h = 2^log_n. */
int lsp_gen_permutation_trace(uint64_t seed, uint32_t log_n, uint32_t ncols, const lsp_fr *alpha,
                              const lsp_fr *delta, int small_values, lsp_fr *rows_out);

/* The same workload shape generated on the device, for sizes where a host
 * trace would hold tens of GiB per rank (bench.py's sharded 2^24-2^26 leg):
 * raw columns a = seeded hash values < 2^252, b = a with rows shuffled by a
 * seeded bijection i -> (mul i + add) mod 2^log_n, then the permutation
 * witness (lsp_witness_permutation) into the row-major device trace of
 * 2^log_n x (2 ncols + 2) elements.  Not the host generator's values (that
 * one uses Fisher-Yates); deterministic in the seed, identical on every rank. */
int lsp_gen_permutation_trace_device(lsp_ctx *ctx, uint64_t seed, uint32_t log_n, uint32_t ncols,
                                     const lsp_fr *alpha, const lsp_fr *delta, lsp_fr *trace_dev);

/* Synthetic wide trace (stand-in for the missing zkevm.bin):
 * nlookup LogUp lookups (RawLookupTrace::get_trace, trace/src/lookup.rs:46-176;
 * A = na columns drawn from ntab tables of na columns) then nperm permutation
 * groups of pcols + pcols columns, laid out as RawTrace::push_traces does
 * (trace/src/lib.rs:62-106).  Call with rows_out == NULL to get the width and
 * the AIR descriptor length; then with buffers of h*width elements and
 * air_len int32s. */
int lsp_gen_wide_trace(uint64_t seed, uint32_t log_n, uint32_t nlookup, uint32_t na, uint32_t ntab, uint32_t nperm,
                       uint32_t pcols, const lsp_fr *alpha, const lsp_fr *delta, lsp_fr *rows_out, size_t rows_cap,
                       int32_t *air_out, size_t air_cap, size_t *width_out, size_t *air_len_out);

#ifdef __cplusplus
}
#endif
#endif /* LSP_H */
