#pragma once
#include <vector>

#include "host.hpp"

namespace lsp {
// coset LDE of an h x w device matrix with per-column shifts -> (h << added_bits) x w bit-reversed rows
void lde_device(lsp_ctx* ctx, const Fr* d_in, size_t h, size_t w, uint32_t added_bits, const Fr* shifts_host,
                Fr* d_out);
// leaves + every layer into `layers` (2*height - 1); returns the root
Fr commit_device(lsp_ctx* ctx, const MatList& m, size_t height, Fr* layers);
lsp_proof* prove_device(lsp_ctx* ctx, const Fr* d_trace, size_t h, size_t w, const Air& air, const Fr* pub,
                        size_t npub);
std::vector<uint8_t> serialize(const lsp_proof& p);
// 0 = accept, otherwise the failing check (host CPU verifier)
int verify_host(const lsp_ctx* ctx, const Air& air, const Fr* pub, size_t npub, const uint8_t* b, size_t n);
}  // namespace lsp
