#pragma once
#include <functional>
#include <vector>

#include "host.hpp"

namespace lsp {
// coset LDE of an h x w device matrix with per-column shifts -> (h << added_bits) x w bit-reversed rows;
// with nk > 0 only the coset blocks [k0, k0 + nk) (rows k0*h .. (k0+nk)*h - 1 of the full result)
void lde_device(lsp_ctx* ctx, const Fr* d_in, size_t h, size_t w, uint32_t added_bits, const Fr* shifts_host,
                Fr* d_out, uint32_t k0 = 0, uint32_t nk = 0);
// TwoAdicSubgroupDft::coset_dft_batch / coset_idft_batch on device matrices (h x w row-major):
// coefficients -> evaluations on shift H_h stored bit-reversed, and natural-order evaluations -> coefficients
void coset_dft_device(lsp_ctx* ctx, const Fr* d_coef, size_t h, size_t w, const Fr& shift, Fr* d_out);
void coset_idft_device(lsp_ctx* ctx, const Fr* d_evals, size_t h, size_t w, const Fr& shift, Fr* d_out);
// leaves + every layer into `layers` (2*height - 1); returns the root
// fold: when set, the leaves are the pairs of the FRI fold it describes (fused
// into the leaf kernel; m.ptr[0] receives the folded vector)
// the pending phase events of the last proof -> ctx->timings (prove.cpp)
void resolve_timings(lsp_ctx* ctx);
// side (optional): called once, after the tree's launches are issued and before
// the host waits for them, with an event on the context's stream that follows
// the leaves and the wide levels (every level of more than 2^15 digests): work
// queued behind it on another stream fills the chip beside the narrow levels
// and the host's tree top
Fr commit_device(lsp_ctx* ctx, const MatList& m, size_t height, Fr* layers, const FoldSpec* fold = nullptr,
                 const std::function<void(hipEvent_t)>* side = nullptr);
lsp_proof* prove_device(lsp_ctx* ctx, const Fr* d_trace, size_t h, size_t w, const Air& air, const Fr* pub,
                        size_t npub);
struct Comm;
// one rank of a proof sharded over comm.size ranks (prove_device = 1 rank);
// every rank returns the same proof
lsp_proof* prove_shard(lsp_ctx* ctx, Comm& comm, const Fr* d_trace, size_t h, size_t w, const Air& air,
                       const Fr* pub, size_t npub);
// collective (every rank of comm): time an allgather of up to 256 MiB and this
// GPU's inverse NTT, agree on the minimum over the ranks (comm.ag_gbs,
// comm.intt_gelem_s; every rank's raw values in comm.calib_raw)
void calibrate_exchange(lsp_ctx* ctx, Comm& comm);
// this GPU's inverse-NTT rate (G elements/s) on an h x w matrix of seeded
// random elements, h = 2^log_h: median of `reps` after a warm-up, `before`
// ahead of each rep (may be empty)
double calibrate_intt(lsp_ctx* ctx, uint32_t log_h, size_t w, int reps, const std::function<void()>& before);
// the quotient-chunk broadcasts a sharded proof of h rows with q chunks issues
// on comm (either exchange choice): their count, bytes each, and their time
// at the calibrated allgather bandwidth (0 when uncalibrated)
struct QuotientExchange {
    size_t bcasts, bytes_each;
    double model_ms;
};
QuotientExchange quotient_exchange(const Comm& comm, size_t h, size_t q, uint32_t log_blowup);
// the inverse-NTT exchange a sharded proof of h x w (q quotient chunks) over
// comm makes: true = split by columns + an allgather of the coefficients,
// false = every rank inverts every column (LSP_SHARD_SPLIT_INTT=0/1 forces
// it); rank-identical
struct ExchangePlan {
    bool split;
    double allgather_ms, redundant_ms;  // the model's two costs (0 when uncalibrated)
    const char* reason;
};
ExchangePlan exchange_plan(const Comm& comm, size_t h, size_t w, size_t q, uint32_t log_blowup);
// proof wire format and field view (proof.cpp)
// pool (optional): the queries are written in parallel (the element
// conversions to canonical words are ~2/3 of a 2^19 proof's 10 K elements)
// reuse (optional): a buffer whose allocation the result takes over
std::vector<uint8_t> serialize(const lsp_proof& p, HostPool* pool = nullptr, std::vector<uint8_t>* reuse = nullptr);
lsp_proof* deserialize(const uint8_t* buf, size_t len);
// A freed proof's largest allocations -- its wire bytes (a fresh 324 KB vector
// per 2^19 proof is an mmap, page faults and an munmap) and its query records
// (~800 small vectors) -- go back to a small process-wide stock that the next
// proof's query assembly and serialization take from (proof.cpp)
void proof_release(lsp_proof* p);
std::vector<uint8_t> recycled_wire();
std::vector<lsp_query> recycled_queries();
void proof_view(const lsp_proof& p, lsp_proof_view* v);
lsp_proof* proof_from_view(const lsp_proof_view& v);
// communicators of a process-per-GPU sharded prove (comm_ext.cpp)
Comm* make_callback_comm(const lsp_comm_ops& ops);
void rccl_unique_id(uint8_t out[128]);
Comm* make_rccl_comm(const uint8_t id[128], int rank, int size);
// witness blocks on the device (witness.cpp): rows written at out + i * ostride
void witness_permutation_device(lsp_ctx* ctx, const Fr* a, uint32_t na, const Fr* b, uint32_t nb, size_t n,
                                const Fr& alpha, const Fr& delta, Fr* out, size_t ostride);
void witness_lookup_device(lsp_ctx* ctx, const Fr* a, uint32_t na, const Fr* b, uint32_t nt, uint32_t nbc,
                           const Fr* afil, const Fr* bfil, size_t n, const Fr& alpha, const Fr& delta, Fr* out,
                           size_t ostride);
// CBOR RawPermutationTrace / RawLookupTrace (cbor.cpp)
lsp_raw_trace* parse_raw_trace(const uint8_t* buf, size_t len);
void raw_trace_shape(const lsp_raw_trace& t, size_t& height, size_t& width);
std::vector<Fr> raw_trace_columns(const lsp_raw_trace& t, size_t height);
// 0 = accept, otherwise the failing check (host CPU verifier)
int verify_host(const lsp_ctx* ctx, const Air& air, const Fr* pub, size_t npub, const uint8_t* b, size_t n);
}  // namespace lsp
