/*
 * lsp_oracle -- plain-C restatement of the reference prover's hot path.
 *
 * TEST INFRASTRUCTURE ONLY: linked/loaded only by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg, as the checker and as the timed CPU
 * baseline ("kind": "port").  The product library never links it.
 *
 * It restates, with 4 x 64-bit Montgomery limbs and unsigned __int128 (a
 * different limb system from the product's 8 x 32-bit device arithmetic), the
 * same algorithm as oracle/pyoracle.py; see that file's header for the
 * reference file:line map and the parity status (conventions U1..U12 are
 * parity unpinned; unique quantities are pinned by theorem).
 *
 * Element format everywhere: uint64_t[4] little-endian Montgomery form,
 * R = 2^256 (ark-ff 0.5 in-memory form).
 */
#ifndef LSP_ORACLE_H
#define LSP_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { uint64_t l[4]; } lo_fr;

typedef struct {
    uint32_t sbox_degree, rounds_f, rounds_p;
    lo_fr ext_initial[8][3];
    lo_fr ext_terminal[8][3];
    lo_fr internal[64];
    lo_fr alpha, delta; /* permutation challenges (public values) */
    /* U2/U3 linear layers: generic_lin == 0 -> the defaults (external
     * circ(2,1,1), internal J + diag(1,1,2)); otherwise s <- ext_mds s
     * (row-major) and s_i <- (s0+s1+s2) + int_diag[i] s_i */
    uint32_t generic_lin;
    lo_fr ext_mds[9];
    lo_fr int_diag[3];
} lo_params;

/* transcript conventions (include/lsp.h lsp_params):
 * lo_fri.transcript is an OR of these, 0 = the defaults */
enum {
    LO_T_SKIP_LOG_DEGREE = 1,    /* U7: log2(h) not observed */
    LO_T_SKIP_PUBLIC = 2,        /* U7: public values not observed before alpha */
    LO_T_OBSERVE_OPENED = 4,     /* U7: opened values observed before alpha_fri */
    LO_T_SAMPLE_BITS_MONT = 8,   /* U8: sample_bits from the Montgomery form */
    LO_T_SKIP_FINAL_POLY = 16    /* U12: final polynomial not observed */
};

typedef struct {
    uint32_t log_blowup, log_final_poly_len, num_queries, pow_bits;
    uint32_t transcript;
} lo_fri;

/* field helpers */
void lo_fr_from_u64(uint64_t x, lo_fr *out);
void lo_fr_to_canonical(const lo_fr *a, uint64_t out[4]);
void lo_fr_from_canonical(const uint64_t in[4], lo_fr *out);
void lo_fr_mul(const lo_fr *a, const lo_fr *b, lo_fr *out);
void lo_fr_add(const lo_fr *a, const lo_fr *b, lo_fr *out);
void lo_fr_inv(const lo_fr *a, lo_fr *out);

/* U4/U5 seeded setup (SplitMix64): alpha, delta, then Poseidon2 constants */
void lo_setup(uint64_t seed, uint32_t sbox_degree, uint32_t rounds_f, uint32_t rounds_p, lo_params *out);

/* primitives */
void lo_poseidon2_permute(const lo_params *p, lo_fr state[3]);
void lo_hash_iter(const lo_params *p, const lo_fr *in, size_t n, lo_fr *out);
void lo_coset_lde_batch(const lo_fr *in, size_t h, size_t w, uint32_t added_bits,
                        const lo_fr *shifts /* w entries */, lo_fr *out, int nthreads);
/* p_c(xs[k]) for the columns of a row-major h x w matrix of values on H_h
 * (barycentric; no NTT); out is npts x w.  lo_lde_point: the point of LDE
 * output row j (bit-reversed over N = h << added_bits, coset `shift`). */
void lo_eval_points(const lo_fr *in, size_t h, size_t w, const lo_fr *xs, size_t npts, lo_fr *out, int nthreads);
void lo_lde_point(size_t h, uint32_t added_bits, const lo_fr *shift, uint64_t j, lo_fr *out);
/* Merkle over k equal-height matrices given as one row-major h x W buffer
 * (W = sum of widths, rows concatenated in commit order). layers_out gets
 * 2h-1 digests: leaves first, root last. */
void lo_merkle_commit(const lo_params *p, const lo_fr *rows, size_t h, size_t W,
                      lo_fr *layers_out, int nthreads);

/* synthetic permutation trace: row-major h x (2*ncols+2) */
int lo_gen_perm_trace(uint32_t log_n, uint32_t ncols, const lo_fr *alpha, const lo_fr *delta,
                      uint64_t seed, int small, lo_fr *rows_out);

/* AIR descriptor: see include/lsp.h (LSP_AIR_*) -- the same int32 encoding */
int lo_log_quotient_degree(const int32_t *air, size_t air_len, int public_degree);

/* Full prove. proof bytes are malloc'd; free with lo_free. dbg (nullable)
 * receives intermediate vectors for parity tests: see lsp_oracle.c. */
typedef struct {
    lo_fr *trace_lde;       /* N*w */
    lo_fr *trace_layers;    /* 2N-1 */
    lo_fr *quotient;        /* Q */
    lo_fr *quotient_lde;    /* N*q */
    lo_fr *quotient_layers; /* 2N-1 */
    lo_fr *fri_input;       /* N */
    lo_fr challenges[4];    /* alpha, zeta, alpha_fri, final_poly */
} lo_debug;

int lo_prove(const lo_params *p, const lo_fri *fri, const lo_fr *trace, size_t h, size_t w,
             const int32_t *air, size_t air_len, int public_degree, int nthreads,
             uint8_t **proof_out, size_t *proof_len, lo_debug *dbg);
int lo_verify(const lo_params *p, const lo_fri *fri, const int32_t *air, size_t air_len,
              int public_degree, const uint8_t *proof, size_t proof_len);
void *lo_alloc(size_t bytes);
void lo_free(void *ptr);

#ifdef __cplusplus
}
#endif
#endif
