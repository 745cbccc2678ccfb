/* The drop-in boundary from plain C: everything below uses only
 * include/lsp.h -- what a Rust -sys crate or any other FFI
 * binds.  bin/src/main.rs's flow: seeded challenges and Poseidon2
 * constants (main.rs:29-31,49), a permutation trace with its witness
 * (trace/src/permutation.rs:24-93), prove (main.rs:80-86), serialize,
 * verify (main.rs:88-96).
 *
 *   prove_c [log_n] [--host-only]
 * --host-only: no GPU -- exercises the host entry points only (setup, field
 * conversions, trace generation, verifier context) and exits 0.  */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lsp.h"

#define CHECK(call, ctx)                                                                     \
    do {                                                                                     \
        int rc_ = (call);                                                                    \
        if (rc_ != LSP_OK) {                                                                 \
            fprintf(stderr, "%s failed: %d (%s)\n", #call, rc_, lsp_last_error(ctx));        \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

int main(int argc, char** argv) {
    uint32_t log_n = 10;
    int host_only = 0;
    for (int i = 1; i < argc; ++i) {
        if (strcmp(argv[i], "--host-only") == 0)
            host_only = 1;
        else
            log_n = (uint32_t)atoi(argv[i]);
    }
    const uint32_t rounds_f = 8, rounds_p = 22, ncols = 3;
    lsp_fr alpha, delta, rc[3 * 8 + 22];
    CHECK(lsp_seeded_setup(0x4C494E4541ull, rounds_f, rounds_p, &alpha, &delta, rc), NULL);

    /* field round trip through the canonical form */
    uint64_t canon[4];
    lsp_fr back;
    lsp_fr_to_canonical(&alpha, canon);
    lsp_fr_from_canonical(canon, &back);
    if (memcmp(&back, &alpha, sizeof back) != 0) {
        fprintf(stderr, "canonical round trip failed\n");
        return 1;
    }

    const size_t h = (size_t)1 << log_n, w = 2 * ncols + 2;
    lsp_fr* trace = (lsp_fr*)malloc(h * w * sizeof(lsp_fr));
    CHECK(lsp_gen_permutation_trace(0x4C494E4541ull, log_n, ncols, &alpha, &delta, 0, trace), NULL);

    /* the AIR: one AirPermutationConfig (air/src/air_permutation.rs:1-24) */
    int32_t air[1 + 3 + 2 * 3 + 2];
    size_t k = 0;
    air[k++] = 1;
    air[k++] = LSP_AIR_PERMUTATION;
    air[k++] = (int32_t)ncols;
    air[k++] = (int32_t)ncols;
    for (uint32_t c = 0; c < 2 * ncols; ++c) air[k++] = (int32_t)c;
    air[k++] = (int32_t)(2 * ncols);
    air[k++] = (int32_t)(2 * ncols + 1);
    uint32_t log_q = 0;
    CHECK(lsp_log_quotient_degree(air, k, 1, &log_q), NULL);

    lsp_params p;
    memset(&p, 0, sizeof p); /* zero = the default transcript conventions (U7/U8/U12) */
    p.struct_size = (uint32_t)sizeof p;
    p.sbox_degree = 11;
    p.rounds_f = rounds_f;
    p.rounds_p = rounds_p;
    p.round_constants = rc;
    p.log_blowup = 3;
    p.log_final_poly_len = 0;
    p.num_queries = 33;
    p.proof_of_work_bits = 0;
    p.public_degree = 1;
    const lsp_fr pub[2] = {alpha, delta};

    if (host_only) {
        lsp_ctx* v = NULL;
        CHECK(lsp_ctx_create(LSP_HOST_ONLY, &p, &v), NULL);
        lsp_proof* pf = NULL;
        const int rc_prove = lsp_prove(v, trace, h, w, air, k, pub, 2, LSP_MEM_HOST, &pf);
        printf("%s: host-only ok (log_q %u, prove on a host-only context -> %d)\n", lsp_version(), log_q, rc_prove);
        lsp_ctx_destroy(v);
        free(trace);
        return rc_prove == LSP_E_STATE ? 0 : 1;
    }

    lsp_ctx* ctx = NULL;
    CHECK(lsp_ctx_create(0, &p, &ctx), NULL);
    lsp_proof* proof = NULL;
    CHECK(lsp_prove(ctx, trace, h, w, air, k, pub, 2, LSP_MEM_HOST, &proof), ctx);
    size_t len = 0;
    CHECK(lsp_proof_serialize(proof, NULL, 0, &len), ctx);
    uint8_t* bytes = (uint8_t*)malloc(len);
    CHECK(lsp_proof_serialize(proof, bytes, len, &len), ctx);
    const int ok = lsp_verify(ctx, air, k, pub, 2, bytes, len);
    /* the proof as p3_uni_stark::Proof<SC> fields (lsp_proof_view) and back to the same bytes */
    lsp_proof_view view;
    CHECK(lsp_proof_get_view(proof, &view), ctx);
    lsp_proof* rebuilt = NULL;
    CHECK(lsp_proof_from_view(&view, &rebuilt), ctx);
    size_t len2 = 0;
    CHECK(lsp_proof_serialize(rebuilt, NULL, 0, &len2), ctx);
    uint8_t* bytes2 = (uint8_t*)malloc(len2);
    CHECK(lsp_proof_serialize(rebuilt, bytes2, len2, &len2), ctx);
    const int same = len2 == len && memcmp(bytes, bytes2, len) == 0;
    printf("proof view: degree_bits %u, width %u, %u quotient chunks, %u queries, %u FRI rounds, paths %u; "
           "rebuilt bytes %s\n", view.degree_bits, view.width, 1u << view.log_quotient_chunks, view.num_queries,
           view.num_fri_rounds, view.input_path_len, same ? "identical" : "DIFFER");
    lsp_proof_free(rebuilt);
    free(bytes2);
    bytes[len / 2] ^= 1;
    const int bad = lsp_verify(ctx, air, k, pub, 2, bytes, len);
    printf("2^%u rows: proof %zu bytes, verify %s, tampered %s\n", log_n, len, ok == LSP_OK ? "ok" : "FAILED",
           bad == LSP_OK ? "ACCEPTED" : "rejected");
    lsp_proof_free(proof);
    lsp_ctx_destroy(ctx);
    free(bytes);
    free(trace);
    return (ok == LSP_OK && bad != LSP_OK && same) ? 0 : 1;
}
