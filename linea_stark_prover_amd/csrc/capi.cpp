// extern "C" entry points of liblsp_hip.so (declared in include/lsp.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <thread>

#include "comm.hpp"
#include "prove_internal.hpp"

using namespace lsp;

namespace {
thread_local std::string g_err;  // errors without a context

#ifdef LSP_DEBUG_BOUNDS
// The debug build: every kernel translation unit's fault word after a C-ABI
// call (dbg_bounds.hpp), with its (file code, line) mapped back to a name
std::string bounds_fault_report() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return "";
    (void)hipDeviceSynchronize();  // the call's kernels are done (any stream)
    static const char* const files[] = {"k_ntt.hip", "k_hash.hip", "k_field.hip", "k_quotient.hip", "k_open.hip",
                                        "k_witness.hip", "fr29.hpp", "k_common.hpp", "poseidon2_f29.hpp", "fr.hpp"};
    static unsigned (*const readers[])() = {bounds_fault_k_ntt, bounds_fault_k_hash, bounds_fault_k_field,
                                            bounds_fault_k_quotient, bounds_fault_k_open, bounds_fault_k_witness};
    static const char* const tus[] = {"k_ntt.hip", "k_hash.hip", "k_field.hip", "k_quotient.hip", "k_open.hip",
                                      "k_witness.hip"};
    std::string out;
    for (size_t t = 0; t < sizeof readers / sizeof readers[0]; ++t) {
        const unsigned v = readers[t]();
        if (!v) continue;
        std::string file = "file#" + std::to_string(v >> 16);
        for (const char* f : files)
            if (dbg::file_code(f) == (v >> 16)) file = f;
        out += (out.empty() ? "" : "; ") + std::string("device bounds check failed at ") + file + ":" +
               std::to_string(v & 0xffffu) + " (kernels of " + tus[t] + ")";
    }
    return out;
}
#endif

}  // namespace

#ifdef LSP_DEBUG_BOUNDS
void lsp::dbg_check_after(const char* what) {
    const std::string bad = bounds_fault_report();
    if (!bad.empty()) throw LspError(LSP_E_STATE, bad + " after " + what);
}
#endif

namespace {
template <class F>
int guarded(lsp_ctx* ctx, F&& f) {
    try {
        f();
#ifdef LSP_DEBUG_BOUNDS
        const std::string bad = bounds_fault_report();
        if (!bad.empty()) throw LspError(LSP_E_STATE, bad);
#endif
        return LSP_OK;
    } catch (const LspError& e) {
        (ctx ? ctx->err : g_err) = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        (ctx ? ctx->err : g_err) = "host allocation failed";
        return LSP_E_OOM;
    } catch (const std::exception& e) {
        (ctx ? ctx->err : g_err) = e.what();
        return LSP_E_STATE;
    }
}

// device input: either the caller's device pointer or a pool copy of host data.
// The host copy is one pageable hipMemcpyAsync: it moves a 2^19 x 8 trace at
// 56 GB/s, the PCIe link's rate -- the same as from pinned memory (57) or from
// the caller's buffer registered in place (57; 27 once the registration of a
// fresh buffer is counted), and faster than staging through a pinned ring
// filled by host threads (37-46): tools/ubench/h2d.hip, profiles/r05b_h2d.json,
// r05c_h2d.json; in-proof A/B tools/time_upload.py, profiles/r05c_time_upload.txt
const Fr* dev_in(lsp_ctx* ctx, const lsp_fr* p, size_t n, int mem, const char* name) {
    LSP_REQUIRE(p || n == 0, LSP_E_ARG, "null input pointer");
    if (mem == LSP_MEM_DEVICE) return reinterpret_cast<const Fr*>(p);
    LSP_REQUIRE(mem == LSP_MEM_HOST, LSP_E_ARG, "mem must be LSP_MEM_HOST or LSP_MEM_DEVICE");
    Fr* d = ctx->fbuf(name, n ? n : 1);
    if (n) LSP_HIP(hipMemcpyAsync(d, p, n * sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
    return d;
}
Fr* dev_out(lsp_ctx* ctx, lsp_fr* p, size_t n, int mem, const char* name) {
    LSP_REQUIRE(p || n == 0, LSP_E_ARG, "null output pointer");
    if (mem == LSP_MEM_DEVICE) return reinterpret_cast<Fr*>(p);
    return ctx->fbuf(name, n ? n : 1);
}
void finish_out(lsp_ctx* ctx, lsp_fr* p, const Fr* d, size_t n, int mem) {
    if (mem == LSP_MEM_HOST && n)
        LSP_HIP(hipMemcpyAsync(p, d, n * sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
}

void need_gpu(lsp_ctx* ctx) {
    LSP_REQUIRE(ctx, LSP_E_ARG, "null ctx");
    LSP_REQUIRE(ctx->device != LSP_HOST_ONLY, LSP_E_STATE, "host-only context (LSP_HOST_ONLY) has no GPU");
    LSP_HIP(hipSetDevice(ctx->device));
}

struct SplitMix64 {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    // U4: 4 words -> 253-bit mask -> reject >= r
    Fr fr() {
        for (;;) {
            Fr c;
            for (int k = 0; k < 4; ++k) {
                uint64_t x = next();
                c.v[2 * k] = (uint32_t)x;
                c.v[2 * k + 1] = (uint32_t)(x >> 32);
            }
            c.v[7] &= (1u << 29) - 1;
            if (fr_words_lt_mod(c)) return fr_from_canonical(c);
        }
    }
    uint64_t below(uint64_t n) {
        const unsigned __int128 two64 = (unsigned __int128)1 << 64;
        const unsigned __int128 lim = two64 - (two64 % n);
        for (;;) {
            uint64_t x = next();
            if ((unsigned __int128)x < lim) return x % n;
        }
    }
};
}  // namespace

extern "C" {

#ifdef LSP_DEBUG_BOUNDS
const char* lsp_version(void) { return "linea_stark_prover_amd 0.1 (gfx950, debug-bounds)"; }
#else
const char* lsp_version(void) { return "linea_stark_prover_amd 0.1 (gfx950)"; }
#endif

int lsp_debug_bounds_probe(lsp_ctx* ctx) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx, LSP_E_ARG, "null ctx");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
#ifndef LSP_DEBUG_BOUNDS
        throw LspError(LSP_E_STATE, "not a debug-bounds build (python -m linea_stark_prover_amd.build --debug-bounds)");
#else
        uint32_t* sink = (uint32_t*)ctx->buf("bounds_probe", 4 * sizeof(uint32_t));
        LSP_HIP(launch_bounds_probe(sink, ctx->stream));
        ctx->sync();  // guarded() then reports the probe's failed check as LSP_E_STATE
#endif
    });
}

int lsp_device_count(int* n) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(n, LSP_E_ARG, "null");
        int c = 0;
        if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
        *n = c;
    });
}

const char* lsp_last_error(const lsp_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int lsp_seeded_setup(uint64_t seed, uint32_t rounds_f, uint32_t rounds_p, lsp_fr* alpha, lsp_fr* delta,
                     lsp_fr* rc) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(alpha && delta && rc && rounds_f % 2 == 0, LSP_E_ARG, "bad seeded_setup arguments");
        SplitMix64 g{seed};
        *alpha = from_fr(g.fr());
        *delta = from_fr(g.fr());
        for (uint32_t i = 0; i < 3 * rounds_f + rounds_p; ++i) rc[i] = from_fr(g.fr());
    });
}

// The scalar helpers return nothing (the reference's field methods cannot
// fail); a null argument makes them a no-op instead of a fault.
void lsp_fr_from_canonical(const uint64_t in[4], lsp_fr* out) {
    if (!in || !out) return;
    lsp_fr t;
    std::memcpy(t.l, in, 32);
    *out = from_fr(fr_from_canonical(to_fr(t)));
}
void lsp_fr_to_canonical(const lsp_fr* in, uint64_t out[4]) {
    if (!in || !out) return;
    lsp_fr t = from_fr(fr_to_canonical(to_fr(*in)));
    std::memcpy(out, t.l, 32);
}
void lsp_fr_from_be_bytes_mod_order(const uint8_t* be, size_t n, lsp_fr* out) {
    if (!out || (!be && n)) return;
    // Horner over bytes: acc = acc * 256 + byte (mod r)
    const Fr b256 = fr_from_u64(256);
    Fr acc = fr_zero();
    for (size_t i = 0; i < n; ++i) acc = fr_add(fr_mul(acc, b256), fr_from_u64(be[i]));
    *out = from_fr(acc);
}
void lsp_fr_mul(const lsp_fr* a, const lsp_fr* b, lsp_fr* out) {
    if (a && b && out) *out = from_fr(fr_mul(to_fr(*a), to_fr(*b))); }
void lsp_fr_inv(const lsp_fr* a, lsp_fr* out) {
    if (a && out) *out = from_fr(fr_inv(to_fr(*a)));
}
void lsp_two_adic_generator(uint32_t bits, lsp_fr* out) {
    if (!out) return;
    if (bits > 47) bits = 47;
    *out = from_fr(host_two_adic_generator(bits));
}

int lsp_ctx_create(int device, const lsp_params* p, lsp_ctx** out) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(p && out && p->round_constants, LSP_E_ARG, "null params");
        LSP_REQUIRE(p->struct_size == sizeof(lsp_params), LSP_E_ARG,
                    "lsp_params.struct_size must be sizeof(lsp_params) of this header (caller built against "
                    "another lsp.h?)");
        LSP_REQUIRE(p->skip_log_degree <= 1 && p->skip_public_values <= 1 && p->observe_opened_values <= 1 &&
                        p->sample_bits_montgomery <= 1 && p->skip_final_poly <= 1,
                    LSP_E_ARG, "transcript switches are 0 or 1");
        LSP_REQUIRE(p->sbox_degree == 11 || p->sbox_degree == 17, LSP_E_ARG, "S-box degree must be 11 or 17");
        LSP_REQUIRE(p->rounds_f >= 2 && p->rounds_f % 2 == 0 && p->rounds_f <= 64 && p->rounds_p <= 256, LSP_E_ARG,
                    "bad round counts");
        LSP_REQUIRE(p->log_blowup >= 1 && p->log_blowup <= 8 && p->num_queries >= 1 && p->num_queries <= 1024 &&
                        p->proof_of_work_bits <= 32 && p->log_final_poly_len <= 8 &&
                        (p->public_degree == 0 || p->public_degree == 1),
                    LSP_E_ARG, "bad FRI parameters");
        auto c = std::make_unique<lsp_ctx>();
        c->device = device;
        c->p2.L = P2Layout{p->rounds_f, p->rounds_p, p->sbox_degree};
        const size_t nround = 3 * p->rounds_f + p->rounds_p;
        const size_t nrc = nround + P2_LIN_N;  // round constants, then M_E [9] and d [3]
        c->p2.rc.resize(nrc);
        for (size_t i = 0; i < nround; ++i) c->p2.rc[i] = to_fr(p->round_constants[i]);
        {
            // U2/U3: caller-set linear layers; the default values are stored
            // too, and gen_lin picks the generic path only when they differ
            static const uint32_t dm[9] = {2, 1, 1, 1, 2, 1, 1, 1, 2}, dd[3] = {1, 1, 2};
            bool gen = false;
            for (int k = 0; k < 9; ++k) {
                const Fr def = fr_from_u64(dm[k]);
                Fr v = def;
                if (p->external_mds) {
                    v = to_fr(p->external_mds[k]);
                    LSP_REQUIRE(fr_words_lt_mod(v), LSP_E_ARG, "external_mds entry not canonical");
                }
                gen |= !fr_eq(v, def);
                c->p2.rc[nround + k] = v;
            }
            for (int k = 0; k < 3; ++k) {
                const Fr def = fr_from_u64(dd[k]);
                Fr v = def;
                if (p->internal_diag) {
                    v = to_fr(p->internal_diag[k]);
                    LSP_REQUIRE(fr_words_lt_mod(v), LSP_E_ARG, "internal_diag entry not canonical");
                }
                gen |= !fr_eq(v, def);
                c->p2.rc[nround + 9 + k] = v;
            }
            c->p2.L.gen_lin = gen ? 1u : 0u;
        }
        if (ifma::available()) ifma::prepare(c->p2.rc, c->p2.rc8);
        if (device != LSP_HOST_ONLY) {  // LSP_HOST_ONLY: verifier-only context, no GPU touched
            int n = 0;
            if (hipGetDeviceCount(&n) != hipSuccess || n == 0) throw LspError(LSP_E_STATE, "no HIP device");
            LSP_REQUIRE(device >= 0 && device < n, LSP_E_ARG, "bad device index");
            LSP_HIP(hipSetDevice(device));
            LSP_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
            int lds = 0;  // LDS per workgroup (gfx950: 160 KiB): what the reduce-rows launch may use
            if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess && lds > 0)
                c->lds_per_block = (size_t)lds;
            LSP_HIP(hipMalloc(&c->rc_dev, nrc * sizeof(Fr)));
            LSP_HIP(hipMemcpy(c->rc_dev, c->p2.rc.data(), nrc * sizeof(Fr), hipMemcpyHostToDevice));
            LSP_HIP(hipMalloc(&c->rc29_dev, nrc * sizeof(F29)));
            LSP_HIP(launch_rc_to_f29(c->rc_dev, c->rc29_dev, (uint32_t)nrc, c->stream));
            LSP_HIP(hipStreamSynchronize(c->stream));
        }
        c->log_blowup = p->log_blowup;
        c->log_final_poly_len = p->log_final_poly_len;
        c->num_queries = p->num_queries;
        c->pow_bits = p->proof_of_work_bits;
        c->public_degree = p->public_degree;
        c->transcript.log_degree = !p->skip_log_degree;
        c->transcript.public_values = !p->skip_public_values;
        c->transcript.opened_values = p->observe_opened_values != 0;
        c->transcript.mont_bits = p->sample_bits_montgomery != 0;
        c->transcript.final_poly = !p->skip_final_poly;
        *out = c.release();
    });
}

int lsp_ctx_destroy(lsp_ctx* ctx) {
    if (!ctx) return LSP_OK;
    delete ctx->comm;
    ctx->comm = nullptr;
    if (ctx->device == LSP_HOST_ONLY) {
        delete ctx;
        return LSP_OK;
    }
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->side_stream) (void)hipStreamSynchronize(ctx->side_stream);
    for (auto& kv : ctx->pool)
        if (kv.second.p) (void)hipFree(kv.second.p);
    for (auto& kv : ctx->hpool)
        if (kv.second.p) (void)hipHostFree(kv.second.p);
    for (auto& kv : ctx->twiddles) (void)hipFree(kv.second);
    for (auto& kv : ctx->stage_ev) (void)hipEventDestroy(kv.second);
    for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
    for (auto& t : ctx->pending_timings) {
        (void)hipEventDestroy(std::get<1>(t));
        (void)hipEventDestroy(std::get<2>(t));
    }
    if (ctx->ev_near) (void)hipEventDestroy(ctx->ev_near);
    if (ctx->ev_top) (void)hipEventDestroy(ctx->ev_top);
    if (ctx->ev_warm) (void)hipEventDestroy(ctx->ev_warm);
    if (ctx->side_stream) {
        (void)hipStreamSynchronize(ctx->side_stream);
        (void)hipEventDestroy(ctx->ev_wide);
        (void)hipEventDestroy(ctx->ev_side);
        (void)hipStreamDestroy(ctx->side_stream);
    }
    if (ctx->rc_dev) (void)hipFree(ctx->rc_dev);
    if (ctx->rc29_dev) (void)hipFree(ctx->rc29_dev);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return LSP_OK;
}

int lsp_synchronize(lsp_ctx* ctx) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx, LSP_E_ARG, "null ctx");
        need_gpu(ctx);
        LSP_HIP(hipDeviceSynchronize());
    });
}

int lsp_dev_alloc(lsp_ctx* ctx, size_t bytes, void** dptr) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && dptr, LSP_E_ARG, "null");
        need_gpu(ctx);
        if (hipMalloc(dptr, bytes ? bytes : 1) != hipSuccess) {
            (void)hipGetLastError();
            throw LspError(LSP_E_OOM, "hipMalloc failed");
        }
    });
}
int lsp_dev_free(lsp_ctx* ctx, void* dptr) {
    return guarded(ctx, [&] {
        need_gpu(ctx);
        LSP_HIP(hipFree(dptr));
    });
}
int lsp_memcpy_h2d(lsp_ctx* ctx, void* dst, const void* src, size_t bytes) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && ((dst && src) || bytes == 0), LSP_E_ARG, "null memcpy argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        LSP_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
        ctx->sync();
    });
}
int lsp_memcpy_d2h(lsp_ctx* ctx, void* dst, const void* src, size_t bytes) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && ((dst && src) || bytes == 0), LSP_E_ARG, "null memcpy argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        LSP_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
        ctx->sync();
    });
}

int lsp_coset_lde_batch_shifts(lsp_ctx* ctx, const lsp_fr* in, size_t h, size_t w, uint32_t added_bits,
                               const lsp_fr* shifts, lsp_fr* out, int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && shifts && w >= 1, LSP_E_ARG, "bad arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        log2_exact(h);
        LSP_REQUIRE(added_bits <= 16, LSP_E_ARG, "added_bits too large");
        const size_t N = h << added_bits;
        std::vector<Fr> sh(w);
        for (size_t c = 0; c < w; ++c) sh[c] = to_fr(shifts[c]);
        const Fr* din = dev_in(ctx, in, h * w, mem, "api_in");
        Fr* dout = dev_out(ctx, out, N * w, mem, "api_out");
        lde_device(ctx, din, h, w, added_bits, sh.data(), dout);
        finish_out(ctx, out, dout, N * w, mem);
    });
}

int lsp_coset_lde_batch(lsp_ctx* ctx, const lsp_fr* in, size_t h, size_t w, uint32_t added_bits,
                        const lsp_fr* shift, lsp_fr* out, int mem) {
    if (!shift || w == 0) return LSP_E_ARG;
    std::vector<lsp_fr> sh(w, *shift);
    return lsp_coset_lde_batch_shifts(ctx, in, h, w, added_bits, sh.data(), out, mem);
}

int lsp_coset_dft_batch(lsp_ctx* ctx, const lsp_fr* coeffs, size_t h, size_t w, const lsp_fr* shift, lsp_fr* out,
                        int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && w >= 1, LSP_E_ARG, "bad dft arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        log2_exact(h);
        const Fr s = shift ? to_fr(*shift) : fr_one();
        const Fr* din = dev_in(ctx, coeffs, h * w, mem, "api_in");
        Fr* dout = dev_out(ctx, out, h * w, mem, "api_out");
        coset_dft_device(ctx, din, h, w, s, dout);
        finish_out(ctx, out, dout, h * w, mem);
    });
}

int lsp_coset_idft_batch(lsp_ctx* ctx, const lsp_fr* evals, size_t h, size_t w, const lsp_fr* shift, lsp_fr* out,
                         int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && w >= 1, LSP_E_ARG, "bad idft arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        log2_exact(h);
        const Fr s = shift ? to_fr(*shift) : fr_one();
        LSP_REQUIRE(!fr_is_zero(fr_to_canonical(s)), LSP_E_ARG, "coset shift must be nonzero");
        const Fr* din = dev_in(ctx, evals, h * w, mem, "api_in");
        Fr* dout = dev_out(ctx, out, h * w, mem, "api_out");
        coset_idft_device(ctx, din, h, w, s, dout);
        finish_out(ctx, out, dout, h * w, mem);
    });
}

int lsp_poseidon2_permute_batch(lsp_ctx* ctx, lsp_fr* states, size_t n, int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx, LSP_E_ARG, "null ctx");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        Fr* d = const_cast<Fr*>(dev_in(ctx, states, 3 * n, mem, "api_in"));
        LSP_HIP(launch_permute(d, n, ctx->rc29_dev, ctx->p2.L, ctx->stream));
        finish_out(ctx, states, d, 3 * n, mem);
    });
}

int lsp_hash_rows(lsp_ctx* ctx, const lsp_fr* rows, size_t n, size_t w, lsp_fr* out, int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx, LSP_E_ARG, "null ctx");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const Fr* din = dev_in(ctx, rows, n * w, mem, "api_in");
        Fr* dout = dev_out(ctx, out, n, mem, "api_out");
        MatList m{};
        m.ptr[0] = din;
        m.width[0] = (uint32_t)w;
        m.n = 1;
        LSP_HIP(launch_hash_rows(m, n, dout, ctx->rc29_dev, ctx->p2.L, ctx->stream));
        finish_out(ctx, out, dout, n, mem);
    });
}

int lsp_merkle_commit(lsp_ctx* ctx, const lsp_fr* const* mats, const size_t* widths, size_t nmats, size_t height,
                      int mem, lsp_fr* root, lsp_tree** tree) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && mats && widths && root && nmats >= 1 && nmats <= 8, LSP_E_ARG,
                    "bad merkle_commit arguments (1..8 matrices)");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        log2_exact(height);
        auto t = std::make_unique<lsp_tree>();
        t->ctx = ctx;
        t->height = height;
        MatList m{};
        m.n = (uint32_t)nmats;
        for (size_t k = 0; k < nmats; ++k) {
            LSP_REQUIRE(widths[k] >= 1 && mats[k], LSP_E_ARG, "bad matrix");
            Fr* d = nullptr;
            LSP_HIP(hipMalloc(&d, height * widths[k] * sizeof(Fr)));
            t->mats.push_back(d);
            t->widths.push_back(widths[k]);
            LSP_HIP(hipMemcpyAsync(d, mats[k], height * widths[k] * sizeof(Fr),
                                   mem == LSP_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                                   ctx->stream));
            m.ptr[k] = d;
            m.width[k] = (uint32_t)widths[k];
        }
        LSP_HIP(hipMalloc(&t->layers, (2 * height - 1) * sizeof(Fr)));
        *root = from_fr(commit_device(ctx, m, height, t->layers));
        if (tree)
            *tree = t.release();
        else {
            for (auto* d : t->mats) (void)hipFree(d);
            (void)hipFree(t->layers);
        }
    });
}

int lsp_merkle_open(const lsp_tree* t, size_t index, lsp_fr* rows_out, lsp_fr* path_out) {
    if (!t) return LSP_E_ARG;
    lsp_ctx* ctx = t->ctx;
    return guarded(ctx, [&] {
        LSP_REQUIRE(index < t->height, LSP_E_ARG, "index out of range");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        // the commit's host-made top layers go up asynchronously on the context's
        // non-blocking stream; the copies below use the null stream
        LSP_HIP(hipStreamSynchronize(ctx->stream));
        size_t o = 0;
        if (rows_out)
            for (size_t k = 0; k < t->mats.size(); ++k) {
                LSP_HIP(hipMemcpy(rows_out + o, t->mats[k] + index * t->widths[k], t->widths[k] * sizeof(Fr),
                                  hipMemcpyDeviceToHost));
                o += t->widths[k];
            }
        if (path_out) {
            size_t off = 0, len = t->height;
            for (uint32_t i = 0; len > 1; ++i) {
                LSP_HIP(hipMemcpy(path_out + i, t->layers + off + ((index >> i) ^ 1), sizeof(Fr),
                                  hipMemcpyDeviceToHost));
                off += len;
                len >>= 1;
            }
        }
    });
}

int lsp_merkle_layer(const lsp_tree* t, uint32_t level, lsp_fr* out) {
    if (!t || !out) return LSP_E_ARG;
    lsp_ctx* ctx = t->ctx;
    return guarded(ctx, [&] {
        size_t off = 0, len = t->height;
        for (uint32_t i = 0; i < level; ++i) {
            LSP_REQUIRE(len > 1, LSP_E_ARG, "level out of range");
            off += len;
            len >>= 1;
        }
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        // on the context's (non-blocking) stream: the host-made top layers are
        // uploaded asynchronously on it by the commit
        LSP_HIP(hipMemcpyAsync(out, t->layers + off, len * sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
        LSP_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int lsp_merkle_verify(const lsp_ctx* ctx, const lsp_fr* root, const size_t* widths, size_t nmats,
                      uint32_t log_height, size_t index, const lsp_fr* rows, const lsp_fr* path) {
    if (!ctx || !root || !widths || !rows || (log_height && !path)) return LSP_E_ARG;
    size_t tot = 0;
    for (size_t k = 0; k < nmats; ++k) tot += widths[k];
    std::vector<Fr> leaf(tot);
    for (size_t i = 0; i < tot; ++i) leaf[i] = to_fr(rows[i]);
    Fr cur = ctx->p2.hash(leaf.data(), tot);
    for (uint32_t i = 0; i < log_height; ++i) {
        const Fr sib = to_fr(path[i]);
        cur = ((index >> i) & 1) ? ctx->p2.compress(sib, cur) : ctx->p2.compress(cur, sib);
    }
    return fr_eq(cur, to_fr(*root)) ? LSP_OK : LSP_E_VERIFY;
}

int lsp_tree_free(lsp_tree* t) {
    if (!t) return LSP_OK;
    if (t->ctx->device != LSP_HOST_ONLY) (void)hipSetDevice(t->ctx->device);
    for (auto* d : t->mats) (void)hipFree(d);
    (void)hipFree(t->layers);
    delete t;
    return LSP_OK;
}

int lsp_fri_fold(lsp_ctx* ctx, const lsp_fr* v, size_t len, const lsp_fr* beta, lsp_fr* out, int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && beta && len >= 2, LSP_E_ARG, "bad fri_fold arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const uint32_t lg = log2_exact(len);
        const size_t m = len / 2;
        const Fr* din = dev_in(ctx, v, len, mem, "api_in");
        Fr* dout = dev_out(ctx, out, m, mem, "api_out");
        const Fr half = fr_inv(fr_from_u64(2));
        const Fr ginv = fr_inv(host_two_adic_generator(lg));
        uint32_t L1 = (lg - 1 + 1) / 2, L2 = (lg - 1) - L1;
        Fr* tab = ctx->fbuf("api_tab", (1ull << L1) + (1ull << L2));
        Fr* b = ctx->fbuf("api_tab_base", 1);
        LSP_HIP(hipMemcpyAsync(b, &ginv, sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
        LSP_HIP(launch_pow_tables(b, 1, L1, L2, nullptr, tab, ctx->stream));
        LSP_HIP(launch_fri_fold(din, m, half, fr_mul(to_fr(*beta), half), tab, L1, dout, ctx->stream));
        finish_out(ctx, out, dout, m, mem);
    });
}

void lsp_fri_fold_row(size_t index, uint32_t log_height, const lsp_fr* beta, const lsp_fr* e0, const lsp_fr* e1,
                      lsp_fr* out) {
    if (!beta || !e0 || !e1 || !out) return;
    const Fr s0 = fr_pow_u64(host_two_adic_generator(log_height + 1), host_bitrev(index, log_height));
    const Fr a = to_fr(*e0), b = to_fr(*e1);
    const Fr r = fr_add(a, fr_mul(fr_mul(fr_sub(to_fr(*beta), s0), fr_sub(b, a)), fr_inv(fr_sub(fr_neg(s0), s0))));
    *out = from_fr(r);
}

int lsp_log_quotient_degree(const int32_t* air, size_t air_len, int32_t public_degree, uint32_t* log_q) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(log_q, LSP_E_ARG, "null");
        *log_q = Air::parse(air, air_len).log_quotient_degree(public_degree);
    });
}

int lsp_quotient_values(lsp_ctx* ctx, const lsp_fr* lde, size_t h, size_t w, const int32_t* air, size_t air_len,
                        const lsp_fr* pubv, size_t npub, const lsp_fr* alpha, lsp_fr* out, int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && alpha && pubv && npub >= 2, LSP_E_ARG, "bad quotient arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const Air A = Air::parse(air, air_len);
        LSP_REQUIRE(A.max_col < w, LSP_E_ARG, "AIR column outside width");
        const uint32_t log_h = log2_exact(h), log_q = A.log_quotient_degree(ctx->public_degree);
        const uint32_t logQ = log_h + log_q;
        LSP_REQUIRE(log_q <= ctx->log_blowup, LSP_E_ARG, "quotient degree exceeds blowup");
        const size_t N = h << ctx->log_blowup, Q = (size_t)1 << logQ, q = (size_t)1 << log_q;
        const Fr* dlde = dev_in(ctx, lde, N * w, mem, "api_in");
        Fr* dout = dev_out(ctx, out, Q, mem, "api_out");
        const Fr GEN = host_generator(), one = fr_one();
        const Fr wh_inv = fr_inv(host_two_adic_generator(log_h));
        uint32_t L1 = (logQ + 1) / 2, L2 = logQ - L1;
        Fr* tab = ctx->fbuf("api_tab", (1ull << L1) + (1ull << L2));
        Fr* b = ctx->fbuf("api_tab_base", 1);
        const Fr gq = host_two_adic_generator(logQ);
        LSP_HIP(hipMemcpyAsync(b, &gq, sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
        LSP_HIP(launch_pow_tables(b, 1, L1, L2, nullptr, tab, ctx->stream));
        Fr* den = ctx->fbuf("q_den", Q);
        Fr* inv_den = ctx->fbuf("q_invden", Q);
        LSP_HIP(launch_selector_denoms(tab, L1, GEN, wh_inv, Q, den, ctx->stream));
        LSP_HIP(launch_batch_inverse(den, inv_den, Q, ctx->stream, ctx->bi_scratch(Q)));
        std::vector<Fr> zz(2 * q);
        const Fr gh = fr_pow_u64(GEN, h), gl = host_two_adic_generator(log_q);
        Fr gg = one;
        for (size_t k = 0; k < q; ++k) {
            zz[k] = fr_sub(fr_mul(gh, gg), one);
            zz[q + k] = fr_inv(zz[k]);
            gg = fr_mul(gg, gl);
        }
        Fr* dz = ctx->fbuf("q_zh", 2 * q);
        LSP_HIP(hipMemcpyAsync(dz, zz.data(), zz.size() * sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
        int32_t* dair = (int32_t*)ctx->buf("air", A.raw.size() * sizeof(int32_t));
        LSP_HIP(hipMemcpyAsync(dair, A.raw.data(), A.raw.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                               ctx->stream));
        QuotientArgs qa;
        qa.lde = dlde;
        qa.w = (uint32_t)w;
        qa.logQ = logQ;
        qa.log_q = log_q;
        qa.air = dair;
        qa.air_len = (uint32_t)A.raw.size();
        qa.pub_alpha = to_fr(pubv[0]);
        qa.pub_delta = to_fr(pubv[1]);
        qa.alpha = to_fr(*alpha);
        qa.gen = GEN;
        qa.wh_inv = wh_inv;
        qa.tabQ = tab;
        qa.L1 = L1;
        qa.zh = dz;
        qa.inv_zh = dz + q;
        qa.inv_den = inv_den;
        qa.out = dout;
        qa.lde_rows = (uint64_t)h << ctx->log_blowup;
        LSP_HIP(launch_quotient(qa, ctx->stream));
        finish_out(ctx, out, dout, Q, mem);
    });
}

int lsp_interpolate_coset(lsp_ctx* ctx, const lsp_fr* lde_bitrev, size_t h, size_t w, const lsp_fr* shift,
                          const lsp_fr* z, lsp_fr* ys_out, int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && shift && z && ys_out && w >= 1, LSP_E_ARG, "bad interpolate arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const uint32_t logh = log2_exact(h);
        const Fr* dm = dev_in(ctx, lde_bitrev, h * w, mem, "api_in");
        const Fr S = to_fr(*shift), Z = to_fr(*z);
        uint32_t L1 = (logh + 1) / 2, L2 = logh - L1;
        Fr* tab = ctx->fbuf("api_tab", (1ull << L1) + (1ull << L2));
        Fr* b = ctx->fbuf("api_tab_base", 1);
        const Fr gh = host_two_adic_generator(logh);
        LSP_HIP(hipMemcpyAsync(b, &gh, sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
        LSP_HIP(launch_pow_tables(b, 1, L1, L2, nullptr, tab, ctx->stream));
        Fr* den = ctx->fbuf("o_den", h);
        Fr* inv = ctx->fbuf("o_invz", h);
        LSP_HIP(launch_open_denoms(Z, S, tab, L1, logh, h, den, ctx->stream));
        LSP_HIP(launch_batch_inverse(den, inv, h, ctx->stream, ctx->bi_scratch(h)));
        Fr* partial = ctx->fbuf("o_partial", ((h + 1023) / 1024) * w);
        Fr* sums = ctx->fbuf("o_sums", w);
        uint32_t nb = 0;
        LSP_HIP(launch_interp_partial(dm, (uint32_t)w, h, inv, S, tab, L1, logh, partial, &nb, ctx->stream));
        LSP_HIP(launch_sum_partials(partial, nb, (uint32_t)w, sums, ctx->stream));
        std::vector<Fr> hs(w);
        LSP_HIP(hipMemcpyAsync(hs.data(), sums, w * sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
        ctx->sync();
        const Fr sh = fr_pow_u64(S, h);
        const Fr f = fr_mul(fr_sub(fr_pow_u64(Z, h), sh), fr_inv(fr_mul(sh, fr_from_u64(h))));
        for (size_t c = 0; c < w; ++c) ys_out[c] = from_fr(fr_mul(hs[c], f));
    });
}

int lsp_host_compress_batch(const lsp_ctx* ctx, const lsp_fr* pairs, size_t n, lsp_fr* out) {
    return guarded(const_cast<lsp_ctx*>(ctx), [&] {
        LSP_REQUIRE(ctx && (pairs || n == 0) && (out || n == 0), LSP_E_ARG, "bad host_compress arguments");
        std::vector<Fr> in(2 * n), o(n);
        for (size_t i = 0; i < 2 * n; ++i) in[i] = to_fr(pairs[i]);
        ctx->p2.compress_range(in.data(), o.data(), 0, n);
        for (size_t i = 0; i < n; ++i) out[i] = from_fr(o[i]);
    });
}

int lsp_host_hash_rows(const lsp_ctx* ctx, const lsp_fr* rows, size_t n, size_t w, lsp_fr* out) {
    return guarded(const_cast<lsp_ctx*>(ctx), [&] {
        LSP_REQUIRE(ctx && w >= 1 && (rows || n == 0) && (out || n == 0), LSP_E_ARG, "bad host_hash_rows arguments");
        std::vector<Fr> in(n * w), o(n);
        for (size_t i = 0; i < n * w; ++i) in[i] = to_fr(rows[i]);
        ctx->p2.hash_range(in.data(), w, o.data(), 0, n);
        for (size_t i = 0; i < n; ++i) out[i] = from_fr(o[i]);
    });
}

int lsp_batch_inverse(lsp_ctx* ctx, const lsp_fr* in, size_t n, lsp_fr* out, int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx, LSP_E_ARG, "null ctx");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const Fr* din = dev_in(ctx, in, n, mem, "api_in");
        Fr* dout = dev_out(ctx, out, n, mem, "api_out");
        LSP_REQUIRE(din != dout, LSP_E_ARG, "batch_inverse cannot run in place");
        LSP_HIP(launch_batch_inverse(din, dout, n, ctx->stream, ctx->bi_scratch(n)));
        finish_out(ctx, out, dout, n, mem);
    });
}

int lsp_inverse_denominators(lsp_ctx* ctx, const lsp_fr* points, size_t npoints, uint32_t log_n, const lsp_fr* shift,
                             lsp_fr* out, int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && points && shift && npoints >= 1, LSP_E_ARG, "bad inverse_denominators arguments");
        LSP_REQUIRE(log_n <= 40, LSP_E_SIZE, "log_n too large");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const size_t N = (size_t)1 << log_n;
        Fr* dout = dev_out(ctx, out, npoints * N, mem, "api_out");
        uint32_t L1 = (log_n + 1) / 2, L2 = log_n - L1;
        Fr* tab = ctx->fbuf("api_tab", (1ull << L1) + (1ull << L2));
        Fr* b = ctx->fbuf("api_tab_base", 1);
        const Fr gN = host_two_adic_generator(log_n);
        LSP_HIP(hipMemcpyAsync(b, &gN, sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
        LSP_HIP(launch_pow_tables(b, 1, L1, L2, nullptr, tab, ctx->stream));
        Fr* den = ctx->fbuf("o_den", npoints * N);
        for (size_t p = 0; p < npoints; ++p)
            LSP_HIP(launch_open_denoms(to_fr(points[p]), to_fr(*shift), tab, L1, log_n, N, den + p * N,
                                       ctx->stream));
        LSP_HIP(launch_batch_inverse(den, dout, npoints * N, ctx->stream, ctx->bi_scratch(npoints * N)));
        finish_out(ctx, out, dout, npoints * N, mem);
    });
}

int lsp_open_reduce(lsp_ctx* ctx, const lsp_fr* mat, size_t n, size_t w, const lsp_fr* inv_denoms, const lsp_fr* ys,
                    size_t npoints, const lsp_fr* alpha, lsp_fr* alpha_pow_offset, lsp_fr* ro, int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && ys && alpha && alpha_pow_offset && ro && npoints >= 1 && w >= 1 && n >= 1, LSP_E_ARG,
                    "bad open_reduce arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const Fr* dm = dev_in(ctx, mat, n * w, mem, "api_in");
        const Fr* dinv = dev_in(ctx, inv_denoms, npoints * n, mem, "api_in2");
        Fr* dro = const_cast<Fr*>(dev_in(ctx, ro, n, mem, "api_out"));
        // host side: alpha^c (c < w), per point the offset and offset * sum_c alpha^c y_c
        const Fr A = to_fr(*alpha);
        std::vector<Fr> apw(w), coef(2 * npoints);
        Fr pw = fr_one();
        for (size_t c = 0; c < w; ++c) {
            apw[c] = pw;
            pw = fr_mul(pw, A);
        }
        Fr off = to_fr(*alpha_pow_offset);
        for (size_t p = 0; p < npoints; ++p) {
            Fr ry = fr_zero();
            for (size_t c = 0; c < w; ++c) ry = fr_add(ry, fr_mul(apw[c], to_fr(ys[p * w + c])));
            coef[p] = off;
            coef[npoints + p] = fr_mul(off, ry);
            off = fr_mul(off, pw);  // pw = alpha^w: the offset advances by the matrix width
        }
        Fr* dc = ctx->fbuf("api_coef", w + 2 * npoints);
        LSP_HIP(hipMemcpyAsync(dc, apw.data(), w * sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
        LSP_HIP(hipMemcpyAsync(dc + w, coef.data(), 2 * npoints * sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
        LSP_HIP(launch_reduce_matrix(dm, n, (uint32_t)w, dc, (uint32_t)npoints, dinv, dc + w, dc + w + npoints, dro,
                                     ctx->stream));
        finish_out(ctx, ro, dro, n, mem);
        *alpha_pow_offset = from_fr(off);
    });
}

int lsp_prove(lsp_ctx* ctx, const lsp_fr* trace, size_t h, size_t w, const int32_t* air, size_t air_len,
              const lsp_fr* pubv, size_t npub, int mem, lsp_proof** out) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && out && pubv, LSP_E_ARG, "bad prove arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const Air A = Air::parse(air, air_len);
        std::vector<Fr> pub(npub);
        for (size_t i = 0; i < npub; ++i) pub[i] = to_fr(pubv[i]);
        const Fr* din = dev_in(ctx, trace, h * w, mem, "trace_in");
        *out = prove_device(ctx, din, h, w, A, pub.data(), npub);
    });
}

// ------------------------------------------------------- sharded prove
struct lsp_group {
    std::vector<lsp_ctx*> ctxs;
};

int lsp_group_create(lsp_ctx* const* ctxs, int n, lsp_group** out) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(ctxs && out && n >= 1 && (n & (n - 1)) == 0, LSP_E_ARG, "a group is 2^b contexts");
        auto* grp = new lsp_group();
        grp->ctxs.assign(ctxs, ctxs + n);
        for (lsp_ctx* c : grp->ctxs) {
            if (!c || c->device == LSP_HOST_ONLY) {
                delete grp;
                throw LspError(LSP_E_ARG, "every group member needs a GPU context");
            }
        }
        // peer access between the distinct devices (xGMI copies of the exchanges)
        for (lsp_ctx* a : grp->ctxs)
            for (lsp_ctx* b : grp->ctxs)
                if (a->device != b->device) {
                    LSP_HIP(hipSetDevice(a->device));
                    int ok = 0;
                    LSP_HIP(hipDeviceCanAccessPeer(&ok, a->device, b->device));
                    if (ok) {
                        hipError_t e = hipDeviceEnablePeerAccess(b->device, 0);
                        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) LSP_HIP(e);
                        (void)hipGetLastError();
                    }
                }
        *out = grp;
    });
}

int lsp_group_destroy(lsp_group* grp) {
    delete grp;
    return LSP_OK;
}

int lsp_prove_group(lsp_group* grp, const lsp_fr* const* traces, size_t h, size_t w, const int32_t* air,
                    size_t air_len, const lsp_fr* pubv, size_t npub, int mem, lsp_proof** out) {
    lsp_ctx* c0 = grp && !grp->ctxs.empty() ? grp->ctxs[0] : nullptr;
    return guarded(c0, [&] {
        LSP_REQUIRE(grp && traces && out && pubv, LSP_E_ARG, "bad prove_group arguments");
        const int G = (int)grp->ctxs.size();
        const Air A = Air::parse(air, air_len);
        std::vector<Fr> pub(npub);
        for (size_t i = 0; i < npub; ++i) pub[i] = to_fr(pubv[i]);
        ThreadGroup tg(G);
        for (int r = 0; r < G; ++r) tg.device[r] = grp->ctxs[r]->device;
        std::vector<lsp_proof*> res(G, nullptr);
        std::vector<int> code(G, LSP_OK);
        std::vector<std::string> msg(G);
        std::vector<std::thread> th;
        for (int r = 0; r < G; ++r) {
            th.emplace_back([&, r] {
                lsp_ctx* ctx = grp->ctxs[r];
                try {
                    std::lock_guard<std::mutex> lk(ctx->mu);
                    need_gpu(ctx);
                    const Fr* din = dev_in(ctx, traces[r], h * w, mem, "trace_in");
                    ThreadComm comm(&tg, r);
                    res[r] = prove_shard(ctx, comm, din, h, w, A, pub.data(), npub);
                } catch (const LspError& e) {
                    code[r] = e.code;
                    msg[r] = e.what();
                    tg.abort();
                } catch (const std::exception& e) {
                    code[r] = LSP_E_STATE;
                    msg[r] = e.what();
                    tg.abort();
                }
            });
        }
        for (auto& t : th) t.join();
        int bad = -1;
        for (int r = 0; r < G && bad < 0; ++r)  // report the first rank that failed on its own
            if (code[r] != LSP_OK && msg[r].find("another rank") == std::string::npos) bad = r;
        for (int r = 0; r < G && bad < 0; ++r)
            if (code[r] != LSP_OK) bad = r;
        if (bad < 0) {
            const std::vector<uint8_t> ref = serialize(*res[0]);
            for (int r = 1; r < G; ++r)
                if (serialize(*res[r]) != ref) {
                    bad = r;
                    code[r] = LSP_E_STATE;
                    msg[r] = "ranks disagree on the proof";
                }
        }
        for (int r = (bad < 0 ? 1 : 0); r < G; ++r) delete res[r];
        if (bad >= 0) throw LspError(code[bad], "rank " + std::to_string(bad) + ": " + msg[bad]);
        *out = res[0];
    });
}

int lsp_ctx_attach_comm_ops(lsp_ctx* ctx, const lsp_comm_ops* ops) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && ops && ops->allgather && ops->bcast, LSP_E_ARG, "bad communicator");
        LSP_REQUIRE(ops->size >= 1 && ops->rank >= 0 && ops->rank < ops->size, LSP_E_ARG, "bad rank / size");
        std::lock_guard<std::mutex> g(ctx->mu);
        delete ctx->comm;
        ctx->comm = make_callback_comm(*ops);
    });
}

int lsp_ctx_attach_loopback(lsp_ctx* ctx, int rank, int size) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && size >= 1 && rank >= 0 && rank < size, LSP_E_ARG, "bad rank / size");
        std::lock_guard<std::mutex> g(ctx->mu);
        delete ctx->comm;
        ctx->comm = new LoopbackComm(rank, size);
    });
}

int lsp_ctx_set_phase_timing(lsp_ctx* ctx, int on, const char* const* only, size_t n_only) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && (n_only == 0 || only), LSP_E_ARG, "null argument");
        std::vector<std::string> names;
        for (size_t i = 0; i < n_only; ++i) {
            LSP_REQUIRE(only[i], LSP_E_ARG, "null phase name");
            names.emplace_back(only[i]);
        }
        std::lock_guard<std::mutex> g(ctx->mu);
        ctx->phase_timing = on != 0;
        ctx->phase_only = std::move(names);
    });
}

int lsp_ctx_mem_stats(lsp_ctx* ctx, size_t* pool_bytes, size_t* device_used, size_t* device_total) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && pool_bytes && device_used && device_total, LSP_E_ARG, "null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        size_t pool = 0;
        for (auto& kv : ctx->pool) pool += kv.second.cap;
        *pool_bytes = pool;
        size_t fr = 0, tot = 0;
        LSP_HIP(hipMemGetInfo(&fr, &tot));
        *device_used = tot - fr;
        *device_total = tot;
    });
}

int lsp_comm_rccl_unique_id(uint8_t id[128]) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(id, LSP_E_ARG, "null id");
        rccl_unique_id(id);
    });
}

int lsp_ctx_attach_rccl(lsp_ctx* ctx, const uint8_t id[128], int rank, int size) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && id && size >= 1 && rank >= 0 && rank < size, LSP_E_ARG, "bad RCCL attach arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        delete ctx->comm;
        ctx->comm = nullptr;
        ctx->comm = make_rccl_comm(id, rank, size);
    });
}

int lsp_comm_selftest(lsp_ctx* ctx) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx, LSP_E_ARG, "null ctx");
        std::lock_guard<std::mutex> g(ctx->mu);
        LSP_REQUIRE(ctx->comm, LSP_E_STATE, "no communicator attached");
        need_gpu(ctx);
        Comm& c = *ctx->comm;
        const size_t n = 1000;  // words per rank, not a multiple of anything in particular
        std::vector<uint32_t> mine(n), got(n * (size_t)c.size);
        for (size_t i = 0; i < n; ++i) mine[i] = (uint32_t)(c.rank + 1) * 2654435761u + (uint32_t)i;
        uint32_t* s = (uint32_t*)ctx->buf("selftest_s", n * 4);
        uint32_t* r = (uint32_t*)ctx->buf("selftest_r", n * 4 * (size_t)c.size);
        LSP_HIP(hipMemcpyAsync(s, mine.data(), n * 4, hipMemcpyHostToDevice, ctx->stream));
        c.allgather(ctx, s, r, n * 4);
        LSP_HIP(hipMemcpyAsync(got.data(), r, got.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
        LSP_HIP(hipStreamSynchronize(ctx->stream));
        for (int k = 0; k < c.size; ++k)
            for (size_t i = 0; i < n; ++i)
                LSP_REQUIRE(got[k * n + i] == (uint32_t)(k + 1) * 2654435761u + (uint32_t)i, LSP_E_STATE,
                            "communicator allgather returned wrong data");
        c.bcast(ctx, s, n * 4, 0);
        LSP_HIP(hipMemcpyAsync(got.data(), s, n * 4, hipMemcpyDeviceToHost, ctx->stream));
        LSP_HIP(hipStreamSynchronize(ctx->stream));
        for (size_t i = 0; i < n; ++i)
            LSP_REQUIRE(got[i] == 2654435761u + (uint32_t)i, LSP_E_STATE, "communicator bcast returned wrong data");
        calibrate_exchange(ctx, c);  // what the sharded proofs' inverse-NTT exchange is chosen on
    });
}

int lsp_comm_exchange_plan(lsp_ctx* ctx, size_t h, size_t w, size_t q, double* allgather_gbs, double* intt_gelem_s,
                           size_t* probe_bytes, int* split, double* allgather_ms, double* redundant_ms) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && split, LSP_E_ARG, "null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        LSP_REQUIRE(ctx->comm, LSP_E_STATE, "no communicator attached");
        const Comm& c = *ctx->comm;
        LSP_REQUIRE(q == 0 || (q & (q - 1)) == 0, LSP_E_ARG, "q must be 0 or a power of two");
        const ExchangePlan p = exchange_plan(c, h, w, q, ctx->log_blowup);
        if (allgather_gbs) *allgather_gbs = c.ag_gbs;
        if (intt_gelem_s) *intt_gelem_s = c.intt_gelem_s;
        if (probe_bytes) *probe_bytes = c.ag_probe_bytes;
        *split = p.split ? 1 : 0;
        if (allgather_ms) *allgather_ms = p.allgather_ms;
        if (redundant_ms) *redundant_ms = p.redundant_ms;
    });
}

int lsp_comm_calibration(lsp_ctx* ctx, double* per_rank, size_t cap, size_t* n) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && n, LSP_E_ARG, "null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        LSP_REQUIRE(ctx->comm, LSP_E_STATE, "no communicator attached");
        const std::vector<double>& raw = ctx->comm->calib_raw;
        *n = raw.size();
        if (per_rank && cap >= raw.size()) std::copy(raw.begin(), raw.end(), per_rank);
    });
}

int lsp_comm_quotient_exchange(lsp_ctx* ctx, size_t h, size_t q, size_t* bcasts, size_t* bytes_each,
                               double* model_ms) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx, LSP_E_ARG, "null ctx");
        std::lock_guard<std::mutex> g(ctx->mu);
        LSP_REQUIRE(ctx->comm, LSP_E_STATE, "no communicator attached");
        LSP_REQUIRE(q == 0 || (q & (q - 1)) == 0, LSP_E_ARG, "q must be 0 or a power of two");
        LSP_REQUIRE(h >= 2 && (h & (h - 1)) == 0, LSP_E_ARG, "h must be a power of two >= 2");
        const QuotientExchange x = quotient_exchange(*ctx->comm, h, q, ctx->log_blowup);
        if (bcasts) *bcasts = x.bcasts;
        if (bytes_each) *bytes_each = x.bytes_each;
        if (model_ms) *model_ms = x.model_ms;
    });
}

int lsp_ctx_host_threads(lsp_ctx* ctx, int* n) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && n, LSP_E_ARG, "null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        *n = (int)ctx->host_pool().size();
    });
}

int lsp_comm_info(lsp_ctx* ctx, int* rank, int* size) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && rank && size, LSP_E_ARG, "null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        LSP_REQUIRE(ctx->comm, LSP_E_STATE, "no communicator attached");
        *rank = ctx->comm->rank;
        *size = ctx->comm->size;
    });
}

int lsp_comm_log(lsp_ctx* ctx, char* ops, size_t* bytes, int* roots, double* ms, const char** tags, size_t cap,
                 size_t* n, double* init_ms) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && n, LSP_E_ARG, "null argument");
        std::lock_guard<std::mutex> g(ctx->mu);
        LSP_REQUIRE(ctx->comm, LSP_E_STATE, "no communicator attached");
        need_gpu(ctx);
        Comm& c = *ctx->comm;
        c.resolve_log();
        *n = c.log.size();
        if (init_ms) *init_ms = c.init_ms;
        for (size_t i = 0; i < c.log.size() && i < cap; ++i) {
            const CommRec& r = c.log[i];
            if (ops) ops[i] = r.op;
            if (bytes) bytes[i] = r.bytes;
            if (roots) roots[i] = r.root;
            if (ms) ms[i] = r.ms;
            if (tags) tags[i] = r.tag.c_str();
        }
    });
}

int lsp_ctx_detach_comm(lsp_ctx* ctx) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx, LSP_E_ARG, "null ctx");
        std::lock_guard<std::mutex> g(ctx->mu);
        delete ctx->comm;
        ctx->comm = nullptr;
    });
}

int lsp_prove_sharded(lsp_ctx* ctx, const lsp_fr* trace, size_t h, size_t w, const int32_t* air, size_t air_len,
                      const lsp_fr* pubv, size_t npub, int mem, lsp_proof** out) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && out && pubv, LSP_E_ARG, "bad prove arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        LSP_REQUIRE(ctx->comm, LSP_E_STATE, "no communicator attached (lsp_ctx_attach_*)");
        need_gpu(ctx);
        const Air A = Air::parse(air, air_len);
        std::vector<Fr> pub(npub);
        for (size_t i = 0; i < npub; ++i) pub[i] = to_fr(pubv[i]);
        const Fr* din = dev_in(ctx, trace, h * w, mem, "trace_in");
        *out = prove_shard(ctx, *ctx->comm, din, h, w, A, pub.data(), npub);
    });
}

int lsp_proof_serialize(const lsp_proof* p, uint8_t* buf, size_t cap, size_t* len) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(p && len, LSP_E_ARG, "null");
        std::lock_guard<std::mutex> g(p->cache_mu);
        if (p->wire.empty()) p->wire = serialize(*p);  // a size query and the copy serialize once
        const std::vector<uint8_t>& b = p->wire;
        *len = b.size();
        if (buf) {
            LSP_REQUIRE(!p->rehearsal, LSP_E_STATE,
                        "a rehearsal (loopback) proof is not a proof: only its size can be queried");
            LSP_REQUIRE(cap >= b.size(), LSP_E_ARG, "buffer too small");
            std::memcpy(buf, b.data(), b.size());
        }
    });
}

int lsp_proof_deserialize(const uint8_t* buf, size_t len, lsp_proof** out) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(buf && out, LSP_E_ARG, "null");
        *out = nullptr;
        *out = deserialize(buf, len);
    });
}

int lsp_proof_get_view(const lsp_proof* p, lsp_proof_view* view) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(p && view, LSP_E_ARG, "null");
        LSP_REQUIRE(!p->rehearsal, LSP_E_STATE, "a rehearsal (loopback) proof is not a proof");
        proof_view(*p, view);
    });
}

int lsp_proof_from_view(const lsp_proof_view* view, lsp_proof** out) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(view && out, LSP_E_ARG, "null");
        *out = nullptr;
        *out = proof_from_view(*view);
    });
}

int lsp_proof_free(lsp_proof* p) {
    proof_release(p);  // its wire bytes and query records are reused by the next proof
    return LSP_OK;
}

int lsp_verify(const lsp_ctx* ctx, const int32_t* air, size_t air_len, const lsp_fr* pubv, size_t npub,
               const uint8_t* proof, size_t len) {
    int rc = LSP_OK;
    int g = guarded(nullptr, [&] {
        LSP_REQUIRE(ctx && pubv && proof, LSP_E_ARG, "bad verify arguments");
        const Air A = Air::parse(air, air_len);
        std::vector<Fr> pub(npub);
        for (size_t i = 0; i < npub; ++i) pub[i] = to_fr(pubv[i]);
        const int v = verify_host(ctx, A, pub.data(), npub, proof, len);
        if (v != 0) {
            g_err = "proof rejected at check " + std::to_string(v);
            rc = LSP_E_VERIFY;
        }
    });
    return g != LSP_OK ? g : rc;
}

int lsp_last_timings(const lsp_ctx* ctx, double* ms, const char** names, size_t cap, size_t* n) {
    if (!ctx || !n) return LSP_E_ARG;
    // resolve_timings writes the context's timing state, which lsp_prove writes
    // too: the context's mutex serialises them (a Rust Ctx is Sync)
    lsp_ctx* c = const_cast<lsp_ctx*>(ctx);
    std::lock_guard<std::mutex> g(c->mu);
    try {
        lsp::resolve_timings(c);  // the events are the context's own
    } catch (...) {
        return LSP_E_HIP;
    }
    *n = ctx->timings.size();
    for (size_t i = 0; i < ctx->timings.size() && i < cap; ++i) {
        if (ms) ms[i] = ctx->timings[i].second;
        if (names) names[i] = ctx->timings[i].first.c_str();
    }
    return LSP_OK;
}

int lsp_last_spans(const lsp_ctx* ctx, const char** lines, size_t cap, size_t* n) {
    if (!ctx || !n) return LSP_E_ARG;
    std::lock_guard<std::mutex> g(const_cast<lsp_ctx*>(ctx)->mu);  // spans are rewritten by lsp_prove
    *n = ctx->spans.size();
    for (size_t i = 0; i < ctx->spans.size() && i < cap; ++i)
        if (lines) lines[i] = ctx->spans[i].c_str();
    return LSP_OK;
}

int lsp_calibrate_fr_mul(lsp_ctx* ctx, double* gmul_per_s) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && gmul_per_s, LSP_E_ARG, "null");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const size_t nth = 256 * 256 * 16;  // 16 blocks of 256 lanes per CU
        const uint32_t iters = 256;
        Fr* out = ctx->fbuf("calib", nth);
        LSP_HIP(launch_calib_mul(out, nth, 8, ctx->stream));  // warm
        hipEvent_t e0, e1;
        LSP_HIP(hipEventCreate(&e0));
        LSP_HIP(hipEventCreate(&e1));
        LSP_HIP(hipEventRecord(e0, ctx->stream));
        LSP_HIP(launch_calib_mul(out, nth, iters, ctx->stream));
        LSP_HIP(hipEventRecord(e1, ctx->stream));
        LSP_HIP(hipEventSynchronize(e1));
        float ms = 0;
        LSP_HIP(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        *gmul_per_s = (double)nth * iters * 4 / (ms * 1e-3) / 1e9;
    });
}

// ------------------------------------------------- witness generation (F1)
extern "C++" {
namespace {
// the block's rows: straight into a device trace, or via a scratch block and a
// strided copy into a host trace
template <class F>
void witness_block(lsp_ctx* ctx, lsp_fr* trace, size_t n, size_t trace_w, size_t col0, size_t bw, int mem, F&& fill) {
    LSP_REQUIRE(trace && col0 + bw <= trace_w, LSP_E_ARG, "witness block outside the trace width");
    if (mem == LSP_MEM_DEVICE) {
        fill(reinterpret_cast<Fr*>(trace) + col0, trace_w);
        return;
    }
    Fr* blk = ctx->fbuf("wit_block", n * bw);
    fill(blk, bw);
    LSP_HIP(hipMemcpy2DAsync(reinterpret_cast<Fr*>(trace) + col0, trace_w * sizeof(Fr), blk, bw * sizeof(Fr),
                             bw * sizeof(Fr), n, hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
}
}  // namespace
}

int lsp_witness_permutation(lsp_ctx* ctx, const lsp_fr* a, uint32_t na, const lsp_fr* b, uint32_t nb, size_t n,
                            const lsp_fr* alpha, const lsp_fr* delta, lsp_fr* trace, size_t trace_w, size_t col0,
                            int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && alpha && delta && na >= 1 && nb >= 1 && n >= 1, LSP_E_ARG, "bad witness arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const Fr* da = dev_in(ctx, a, (size_t)na * n, mem, "wit_a");
        const Fr* db = dev_in(ctx, b, (size_t)nb * n, mem, "wit_b");
        const Fr al = to_fr(*alpha), de = to_fr(*delta);
        witness_block(ctx, trace, n, trace_w, col0, (size_t)na + nb + 2, mem, [&](Fr* out, size_t stride) {
            witness_permutation_device(ctx, da, na, db, nb, n, al, de, out, stride);
        });
    });
}

int lsp_gen_permutation_trace_device(lsp_ctx* ctx, uint64_t seed, uint32_t log_n, uint32_t ncols,
                                     const lsp_fr* alpha, const lsp_fr* delta, lsp_fr* trace) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && alpha && delta && trace && ncols >= 1 && log_n >= 1 && log_n <= 30, LSP_E_ARG,
                    "bad device trace-generator arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const size_t n = (size_t)1 << log_n;
        Fr* a = ctx->fbuf("gen_a", (size_t)ncols * n);
        Fr* b = ctx->fbuf("gen_b", (size_t)ncols * n);
        // the row bijection i -> (mul i + add) mod n: mul odd, both from the seed
        const uint64_t mul = ((seed * 0xD1B54A32D192ED03ull) ^ 0x5851F42D4C957F2Dull) | 1u;
        const uint64_t add = seed * 0xA24BAED4963EE407ull + 0x9FB21C651E98DF25ull;
        LSP_HIP(launch_gen_raw_perm(seed, n, ncols, mul, add, a, b, ctx->stream));
        witness_permutation_device(ctx, a, ncols, b, ncols, n, to_fr(*alpha), to_fr(*delta), (Fr*)trace,
                                   2 * (size_t)ncols + 2);
        ctx->release("gen_");
        ctx->release("wit_");
    });
}

int lsp_witness_lookup(lsp_ctx* ctx, const lsp_fr* a, uint32_t na, const lsp_fr* b, uint32_t ntables, uint32_t nbc,
                       const lsp_fr* a_filter, const lsp_fr* b_filter, size_t n, const lsp_fr* alpha,
                       const lsp_fr* delta, lsp_fr* trace, size_t trace_w, size_t col0, int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && alpha && delta && na >= 1 && ntables >= 1 && nbc >= 1 && n >= 1, LSP_E_ARG,
                    "bad witness arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const Fr* da = dev_in(ctx, a, (size_t)na * n, mem, "wit_a");
        const Fr* db = dev_in(ctx, b, (size_t)ntables * nbc * n, mem, "wit_b");
        const Fr* daf = dev_in(ctx, a_filter, n, mem, "wit_af");
        const Fr* dbf = dev_in(ctx, b_filter, (size_t)ntables * n, mem, "wit_bf");
        const Fr al = to_fr(*alpha), de = to_fr(*delta);
        const size_t bw = (size_t)na + (size_t)ntables * (nbc + 3) + 3;
        witness_block(ctx, trace, n, trace_w, col0, bw, mem, [&](Fr* out, size_t stride) {
            witness_lookup_device(ctx, da, na, db, ntables, nbc, daf, dbf, n, al, de, out, stride);
        });
    });
}

// ------------------------------------------------------ trace input (F4)
int lsp_raw_trace_parse(const uint8_t* cbor, size_t len, lsp_raw_trace** out) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(cbor && out, LSP_E_ARG, "null input");
        *out = parse_raw_trace(cbor, len);
    });
}

int lsp_raw_trace_shape(const lsp_raw_trace* t, int* kind, uint32_t* na, uint32_t* ntables, uint32_t* nbc,
                        size_t* max_height, size_t* width) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(t, LSP_E_ARG, "null trace");
        size_t h, w;
        raw_trace_shape(*t, h, w);
        if (kind) *kind = t->kind;
        if (na) *na = (uint32_t)t->a.size();
        if (ntables) *ntables = t->ntables;
        if (nbc) *nbc = t->nbc;
        if (max_height) *max_height = h;
        if (width) *width = w;
    });
}

int lsp_raw_trace_columns(const lsp_raw_trace* t, size_t height, lsp_fr* out, size_t cap, size_t* n) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(t && n, LSP_E_ARG, "null argument");
        const std::vector<Fr> cols = raw_trace_columns(*t, height);
        *n = cols.size();
        if (out) {
            LSP_REQUIRE(cap >= cols.size(), LSP_E_ARG, "buffer too small");
            std::memcpy(out, cols.data(), cols.size() * sizeof(Fr));
        }
    });
}

int lsp_raw_trace_push(lsp_ctx* ctx, const lsp_raw_trace* t, size_t height, const lsp_fr* alpha, const lsp_fr* delta,
                       lsp_fr* trace, size_t trace_w, size_t col0, int mem) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && t && alpha && delta && height >= 1, LSP_E_ARG, "bad raw trace push arguments");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        const std::vector<Fr> cols = raw_trace_columns(*t, height);  // RawTrace resize: zero words
        Fr* d = ctx->fbuf("raw_cols", cols.size());
        LSP_HIP(hipMemcpyAsync(d, cols.data(), cols.size() * sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
        const Fr al = to_fr(*alpha), de = to_fr(*delta);
        const uint32_t na = (uint32_t)t->a.size();
        size_t h, w;
        raw_trace_shape(*t, h, w);
        if (t->kind == LSP_AIR_PERMUTATION) {
            const uint32_t nb = (uint32_t)t->b.size();
            witness_block(ctx, trace, height, trace_w, col0, w, mem, [&](Fr* out, size_t stride) {
                witness_permutation_device(ctx, d, na, d + (size_t)na * height, nb, height, al, de, out, stride);
            });
        } else {
            const Fr* b = d + (size_t)na * height;
            const Fr* af = b + (size_t)t->ntables * t->nbc * height;
            const Fr* bf = af + height;
            witness_block(ctx, trace, height, trace_w, col0, w, mem, [&](Fr* out, size_t stride) {
                witness_lookup_device(ctx, d, na, b, t->ntables, t->nbc, af, bf, height, al, de, out, stride);
            });
        }
        ctx->sync();  // `cols` must outlive the upload
    });
}

int lsp_raw_trace_free(lsp_raw_trace* t) {
    delete t;
    return LSP_OK;
}

int lsp_calibrate_poseidon2(lsp_ctx* ctx, double* mperm_per_s) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && mperm_per_s, LSP_E_ARG, "null");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        // the peak: best of several grid sizes (2..32 blocks of 256 lanes per CU)
        const uint32_t iters = 4;
        Fr* out = ctx->fbuf("calib", (size_t)256 * 256 * 32);
        LSP_HIP(launch_calib_perm(out, (size_t)256 * 256 * 4, 1, ctx->rc29_dev, ctx->p2.L, ctx->stream));  // warm
        hipEvent_t e0, e1;
        LSP_HIP(hipEventCreate(&e0));
        LSP_HIP(hipEventCreate(&e1));
        double best = 0;
        for (size_t per_cu : {2, 4, 8, 16, 32}) {
            const size_t nth = (size_t)256 * 256 * per_cu;
            LSP_HIP(hipEventRecord(e0, ctx->stream));
            LSP_HIP(launch_calib_perm(out, nth, iters, ctx->rc29_dev, ctx->p2.L, ctx->stream));
            LSP_HIP(hipEventRecord(e1, ctx->stream));
            LSP_HIP(hipEventSynchronize(e1));
            float ms = 0;
            LSP_HIP(hipEventElapsedTime(&ms, e0, e1));
            best = std::max(best, (double)nth * iters / (ms * 1e-3) / 1e6);
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        *mperm_per_s = best;
    });
}

int lsp_calibrate_intt(lsp_ctx* ctx, uint32_t log_h, size_t w, double* gelem_per_s) {
    return guarded(ctx, [&] {
        LSP_REQUIRE(ctx && gelem_per_s, LSP_E_ARG, "null argument");
        LSP_REQUIRE(log_h >= 1 && log_h <= 26 && w >= 1 && w <= 1024 && (w << log_h) <= ((size_t)1 << 28), LSP_E_ARG,
                    "bad inverse-NTT probe shape (at most 2^28 elements)");
        std::lock_guard<std::mutex> g(ctx->mu);
        need_gpu(ctx);
        *gelem_per_s = calibrate_intt(ctx, log_h, w, 5, nullptr);
        ctx->release("calib_intt_");
    });
}

int lsp_gen_permutation_trace(uint64_t seed, uint32_t log_n, uint32_t ncols, const lsp_fr* alpha,
                              const lsp_fr* delta, int small_values, lsp_fr* rows) {
    return guarded(nullptr, [&] {
        LSP_REQUIRE(alpha && delta && rows && ncols >= 1 && log_n >= 1 && log_n <= 30, LSP_E_ARG,
                    "bad trace arguments");
        const size_t n = (size_t)1 << log_n, w = 2 * (size_t)ncols + 2;
        SplitMix64 g{seed ^ 0x5452414345ull};  // "TRACE"
        std::vector<Fr> a((size_t)ncols * n);
        for (uint32_t c = 0; c < ncols; ++c)
            for (size_t i = 0; i < n; ++i)
                a[c * n + i] = small_values ? fr_from_u64(g.next() & 0xFFFFFFFFull) : g.fr();
        std::vector<size_t> perm(n);
        for (size_t i = 0; i < n; ++i) perm[i] = i;
        for (size_t i = n - 1; i > 0; --i) std::swap(perm[i], perm[g.below(i + 1)]);
        const Fr al = to_fr(*alpha), dl = to_fr(*delta);
        std::vector<Fr> den(n), inv(n);
        for (size_t i = 0; i < n; ++i) {
            Fr bc = fr_zero();
            for (uint32_t c = 0; c < ncols; ++c) bc = fr_add(fr_mul(bc, al), a[c * n + perm[i]]);
            den[i] = fr_add(bc, dl);
        }
        // batch inverse (RawPermutationTrace::get_trace inverts per row; same values)
        Fr acc = fr_one();
        for (size_t i = 0; i < n; ++i) {
            inv[i] = acc;
            acc = fr_mul(acc, den[i]);
        }
        Fr ia = fr_inv(acc);
        for (size_t i = n; i-- > 0;) {
            const Fr t = fr_mul(ia, inv[i]);
            ia = fr_mul(ia, den[i]);
            inv[i] = t;
        }
        Fr prev = fr_one();
        for (size_t i = 0; i < n; ++i) {
            Fr* row = reinterpret_cast<Fr*>(rows) + i * w;
            Fr ac = fr_zero();
            for (uint32_t c = 0; c < ncols; ++c) {
                row[c] = a[c * n + i];
                row[ncols + c] = a[c * n + perm[i]];
                ac = fr_add(fr_mul(ac, al), row[c]);
            }
            row[2 * ncols] = inv[i];
            prev = fr_mul(fr_mul(prev, fr_add(ac, dl)), inv[i]);
            row[2 * ncols + 1] = prev;
        }
        LSP_REQUIRE(fr_eq(prev, fr_one()), LSP_E_STATE,
                    "failed to check constrain: check column should be 1 on the last row");
    });
}

}  // extern "C"
