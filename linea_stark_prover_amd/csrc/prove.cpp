// Device pipelines (coset LDE, Merkle commit, quotient, open, FRI) and the
// p3_uni_stark::prove orchestration (bin/src/main.rs:80-86) on one GPU.
// The Fiat-Shamir transcript stays on the host (a few dozen hashes); every
// bulk step runs on the device and only roots, opened values and query
// openings cross PCIe.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "comm.hpp"
#include "host.hpp"
#include "prove_internal.hpp"

namespace lsp {

namespace {
// HIP events around each phase (span names as in the reference's bench.log),
// taken from and returned to the context's event pool: creating and destroying
// ~40 events per proof cost ~60 us of host time at the end of every proof
// Phase events are skipped when the context's phase_timing is off
// (lsp_ctx_set_phase_timing) or LSP_PHASE_EVENTS=0, and for phases outside
// the context's phase_only list when it has one; lsp_last_timings reports the
// phases that were timed
struct PhaseTimer {
    lsp_ctx* ctx;
    bool on;
    std::vector<std::pair<std::string, hipEvent_t>> starts;
    std::vector<std::tuple<std::string, hipEvent_t, hipEvent_t>> done;
    explicit PhaseTimer(lsp_ctx* c) : ctx(c) {
        const char* e = std::getenv("LSP_PHASE_EVENTS");
        on = c->phase_timing && !(e && *e == '0');
    }
    hipEvent_t take() {
        hipEvent_t e;
        if (!ctx->event_pool.empty()) {
            e = ctx->event_pool.back();
            ctx->event_pool.pop_back();
        } else {
            LSP_HIP(hipEventCreate(&e));
        }
        return e;
    }
    bool wanted(const std::string& name) const {
        if (!on) return false;
        if (ctx->phase_only.empty()) return true;
        for (const auto& n : ctx->phase_only)
            if (n == name) return true;
        return false;
    }
    void begin(const std::string& name) {
        if (!wanted(name)) return;
        const hipEvent_t e = take();
        LSP_HIP(hipEventRecord(e, ctx->stream));
        starts.emplace_back(name, e);
    }
    void end(const std::string& name) {
        if (!wanted(name)) return;
        for (size_t i = starts.size(); i-- > 0;) {
            if (starts[i].first == name) {
                const hipEvent_t e = take();
                LSP_HIP(hipEventRecord(e, ctx->stream));
                done.emplace_back(name, starts[i].second, e);
                starts.erase(starts.begin() + i);
                return;
            }
        }
    }
    // hand the phase events over for resolve_timings (no wait here: ~40 us of
    // event queries at the end of every proof otherwise)
    void collect() {
        resolve_timings(ctx);  // a previous proof's, if nobody asked for them
        ctx->timings.clear();
        ctx->pending_timings = std::move(done);
        for (auto& st : starts) ctx->event_pool.push_back(st.second);
        done.clear();
        starts.clear();
    }
};

}  // namespace

void resolve_timings(lsp_ctx* ctx) {
    if (ctx->pending_timings.empty()) return;
    ctx->timings.clear();
    for (auto& t : ctx->pending_timings) {
        LSP_HIP(hipEventSynchronize(std::get<2>(t)));
        float ms = 0;
        LSP_HIP(hipEventElapsedTime(&ms, std::get<1>(t), std::get<2>(t)));
        ctx->timings.emplace_back(std::get<0>(t), (double)ms);
        ctx->event_pool.push_back(std::get<1>(t));
        ctx->event_pool.push_back(std::get<2>(t));
    }
    ctx->pending_timings.clear();
}

namespace {
void two_level(uint32_t bits, uint32_t& L1, uint32_t& L2) {
    L1 = (bits + 1) / 2;
    L2 = bits - L1;
}

// two-level power table of `base` covering exponents < 2^bits, in pool buffer `name`
// cached per (base, bits) in the context: the tables of one proof shape (the
// quotient and LDE domains, every FRI round's w^-1) are the same every proof
const Fr* pow_table(lsp_ctx* ctx, const std::string& name, const Fr& base, uint32_t bits, uint32_t& L1) {
    uint32_t L2;
    two_level(bits, L1, L2);
    char key[96];
    std::snprintf(key, sizeof key, "ptab_%u_%08x%08x%08x%08x%08x%08x%08x%08x", bits, base.v[7], base.v[6], base.v[5],
                  base.v[4], base.v[3], base.v[2], base.v[1], base.v[0]);
    auto it = ctx->ptabs.find(key);
    if (it != ctx->ptabs.end()) return it->second;
    Fr* tab = ctx->fbuf(key, (1ull << L1) + (1ull << L2));
    Fr* b = ctx->fbuf(name + "_base", 1);
    LSP_HIP(hipMemcpyAsync(b, &base, sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
    LSP_HIP(launch_pow_tables(b, 1, L1, L2, nullptr, tab, ctx->stream));
    LSP_HIP(hipStreamSynchronize(ctx->stream));  // `base` is a host temporary
    ctx->ptabs[key] = tab;
    return tab;
}

Fr d2h_fr(lsp_ctx* ctx, const Fr* d) {
    Fr x;
    LSP_HIP(hipMemcpyAsync(&x, d, sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
    LSP_HIP(hipStreamSynchronize(ctx->stream));
    return x;
}
}  // namespace

// ----------------------------------------------------------------- LDE
// The twist tables of coset blocks [k0, k0 + nk) of an h x w LDE: coset k,
// column c has base s = shift_c * w_N^bitrev(k); coefficient i is scaled by
// s^i / h (s^i with div_h false: a transform of true coefficients).  Built
// once per (log h, cosets, shifts, div_h) and kept in the context.
struct TwistTables {
    const Fr* tabs;
    uint32_t L1, L2;
    bool shared;  // one table per coset (every column's shift is the same)
};
static TwistTables lde_twist(lsp_ctx* ctx, size_t h, size_t w, uint32_t added_bits, const Fr* shifts_host, uint32_t k0,
                             uint32_t nk, bool div_h = true) {
    const uint32_t logh = log2_exact(h);
    const uint32_t logN = logh + added_bits;
    hipStream_t st = ctx->stream;
    TwistTables T;
    T.shared = true;
    for (size_t c = 1; c < w; ++c) T.shared = T.shared && fr_eq(shifts_host[c], shifts_host[0]);
    const size_t per_coset = T.shared ? 1 : w;
    two_level(logh, T.L1, T.L2);
    const size_t per = (1ull << T.L1) + (1ull << T.L2);
    const size_t nb = (size_t)nk * per_coset;
    uint64_t hsh = 1469598103934665603ull;  // FNV-1a over the shifts' words
    for (size_t c = 0; c < per_coset; ++c)
        for (int i = 0; i < 8; ++i) hsh = (hsh ^ shifts_host[c].v[i]) * 1099511628211ull;
    char key[112];
    std::snprintf(key, sizeof key, "ldetw_%u_%u_%u_%u_%zu_%d_%016llx", logh, added_bits, k0, nk, per_coset,
                  div_h ? 1 : 0, (unsigned long long)hsh);
    auto it = ctx->ptabs.find(key);
    if (it != ctx->ptabs.end()) {
        T.tabs = it->second;
        return T;
    }
    const Fr wN = host_two_adic_generator(logN);
    const Fr hinv = div_h ? host_inv_cached(fr_from_u64(h)) : fr_one();
    std::vector<Fr> bases(2 * nb, hinv);  // nb bases, then nb scales (1/h or 1)
    for (uint32_t k = 0; k < nk; ++k) {
        const Fr ck = fr_pow_u64(wN, host_bitrev(k0 + k, added_bits));
        for (size_t c = 0; c < per_coset; ++c) bases[k * per_coset + c] = fr_mul(shifts_host[c], ck);
    }
    Fr* dbases = ctx->fbuf("lde_bases", 2 * nb);
    ctx->h2d_async("lde_bases_h", dbases, bases.data(), bases.size() * sizeof(Fr));
    const bool keep = ctx->ptabs.size() < 256;  // API callers with ever new shifts: a scratch table
    Fr* t = ctx->fbuf(keep ? key : "lde_tabs", per * nb);
    LSP_HIP(launch_pow_tables(dbases, nb, T.L1, T.L2, dbases + nb, t, st));
    LSP_HIP(launch_to_f29form(t, t, per * nb, st));  // the NTT multiplies by 29-bit-form factors
    if (keep) ctx->ptabs[key] = t;
    T.tabs = t;
    return T;
}

// The chained twist of the fused LDE pass (launch_lde's `ratio`): blocks
// k0 + bitrev_a(j), j < nk = 2^a, k0 a multiple of nk, have the shifts
// shift_c w_N^bitrev_b(k0) rho^j with rho = w_N^(2^b / nk), so the pass twists
// block 0 from its table and every later block by rho^row.  The two-level table
// of rho^i (29-bit form, cached in the context), or nullptr when the range is
// not such a run or LSP_NTT_CHAIN=0 (A/B).
static const Fr* chain_ratio(lsp_ctx* ctx, uint32_t logh, uint32_t added_bits, uint32_t k0, uint32_t nk) {
    static const bool on = [] {
        const char* e = std::getenv("LSP_NTT_CHAIN");
        return !(e && *e == '0');
    }();
    if (!on || logh == 0 || nk < 2 || (nk & (nk - 1)) != 0 || k0 % nk != 0 || nk > (1u << added_bits)) return nullptr;
    const uint32_t logN = logh + added_bits;
    const Fr rho = fr_pow_u64(host_two_adic_generator(logN), (1ull << added_bits) / nk);
    uint32_t L1, L2;
    two_level(logh, L1, L2);
    char key[112];
    std::snprintf(key, sizeof key, "ldechain_%u_%08x%08x%08x%08x%08x%08x%08x%08x", logh, rho.v[7], rho.v[6], rho.v[5],
                  rho.v[4], rho.v[3], rho.v[2], rho.v[1], rho.v[0]);
    auto it = ctx->ptabs.find(key);
    if (it != ctx->ptabs.end()) return it->second;
    Fr* tab = ctx->fbuf(key, (1ull << L1) + (1ull << L2));
    Fr* b = ctx->fbuf("ldechain_base", 1);
    LSP_HIP(hipMemcpyAsync(b, &rho, sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
    LSP_HIP(launch_pow_tables(b, 1, L1, L2, nullptr, tab, ctx->stream));
    LSP_HIP(launch_to_f29form(tab, tab, (1ull << L1) + (1ull << L2), ctx->stream));
    LSP_HIP(hipStreamSynchronize(ctx->stream));  // `rho` is a host temporary
    ctx->ptabs[key] = tab;
    return tab;
}

// Coset blocks [k0, k0 + nk) of the bit-reversed LDE (nk = 0: all
// 2^added_bits): block k = rows k*h .. (k+1)*h - 1 of the full LDE, the
// evaluations on shift_c * w_N^bitrev(k) * H_h.  d_out receives nk blocks.
void lde_device(lsp_ctx* ctx, const Fr* d_in, size_t h, size_t w, uint32_t added_bits, const Fr* shifts_host,
                Fr* d_out, uint32_t k0, uint32_t nk) {
    const uint32_t logh = log2_exact(h);
    const uint32_t B = 1u << added_bits;
    if (nk == 0) nk = B;
    LSP_REQUIRE(k0 + nk <= B, LSP_E_ARG, "coset range outside the LDE");
    LSP_REQUIRE(logh + added_bits <= 47, LSP_E_SIZE, "LDE larger than the 2-adic subgroup");
    Fr* X = ctx->fbuf("lde_X", h * w);
    // with the chained twist the fused pass reads only block k0's table (the
    // later blocks multiply by rho^row), so only that one is built and cached
    const Fr* ratio = chain_ratio(ctx, logh, added_bits, k0, nk);
    const TwistTables T = lde_twist(ctx, h, w, added_bits, shifts_host, k0, ratio ? 1 : nk);
    LSP_HIP(launch_lde(d_in, X, d_out, w, logh, nk, ctx->twiddle29(logh, true), ctx->twiddle29(logh, false), T.tabs,
                       T.L1, T.L2, T.shared ? 0 : 1, ratio, ctx->stream));
}

// The same blocks from h * coefficients (natural order) at `coef`, laid out
// as `map` says -- the forward half, for ranks that split the inverse
static void lde_coeffs_device(lsp_ctx* ctx, const Fr* coef, ColMap map, size_t h, size_t w, uint32_t added_bits,
                              const Fr* shifts_host, Fr* d_out, uint32_t k0, uint32_t nk, bool div_h = true) {
    const uint32_t logh = log2_exact(h);
    LSP_REQUIRE(k0 + nk <= (1u << added_bits) && logh >= 1, LSP_E_ARG, "coset range outside the LDE");
    const Fr* ratio = chain_ratio(ctx, logh, added_bits, k0, nk);  // (block k0's table only, as lde_device)
    const TwistTables T = lde_twist(ctx, h, w, added_bits, shifts_host, k0, ratio ? 1 : nk, div_h);
    LSP_HIP(launch_lde_coeffs(coef, map, d_out, w, logh, nk, ctx->twiddle29(logh, false), T.tabs, T.L1, T.L2,
                              T.shared ? 0 : 1, ratio, ctx->stream));
}

// TwoAdicSubgroupDft::coset_dft_batch ([EXT p3-dft]; dft_batch: shift 1): the
// h x w true coefficients at d_coef -> evaluations on shift H_h, stored
// bit-reversed (row j = p(shift w_h^bitrev(j)), Radix2DitParallel's
// Evaluations layout) -- the forward half of the LDE with one block and
// twist s^i instead of s^i / h
void coset_dft_device(lsp_ctx* ctx, const Fr* d_coef, size_t h, size_t w, const Fr& shift, Fr* d_out) {
    const uint32_t logh = log2_exact(h);
    LSP_REQUIRE(logh <= 40, LSP_E_SIZE, "transform too large");
    if (h == 1) {  // p(x) = c_0 everywhere
        if (d_out != d_coef)
            LSP_HIP(hipMemcpyAsync(d_out, d_coef, w * sizeof(Fr), hipMemcpyDeviceToDevice, ctx->stream));
        return;
    }
    const std::vector<Fr> sh(w, shift);
    lde_coeffs_device(ctx, d_coef, ColMap::plain((uint32_t)w), h, w, 0, sh.data(), d_out, 0, 1, false);
}

// TwoAdicSubgroupDft::coset_idft_batch (idft_batch: shift 1): evaluations on
// shift H_h in natural row order -> the coefficients (natural order,
// canonical): the LDE's inverse half (h c_i), then c_i = X_i (1/h) shift^-i
void coset_idft_device(lsp_ctx* ctx, const Fr* d_evals, size_t h, size_t w, const Fr& shift, Fr* d_out) {
    const uint32_t logh = log2_exact(h);
    LSP_REQUIRE(logh <= 40, LSP_E_SIZE, "transform too large");
    LSP_REQUIRE(!fr_is_zero(fr_to_canonical(shift)), LSP_E_ARG, "coset shift must be nonzero");
    uint32_t L1, L2;
    two_level(logh, L1, L2);
    const size_t per = (1ull << L1) + (1ull << L2);
    Fr* tab = ctx->fbuf("idft_tab", per);
    Fr* b = ctx->fbuf("idft_tab_base", 2);
    const Fr base_scale[2] = {host_inv_cached(shift), host_inv_cached(fr_from_u64(h))};
    LSP_HIP(hipMemcpyAsync(b, base_scale, sizeof base_scale, hipMemcpyHostToDevice, ctx->stream));
    LSP_HIP(launch_pow_tables(b, 1, L1, L2, b + 1, tab, ctx->stream));
    LSP_HIP(launch_to_f29form(tab, tab, per, ctx->stream));
    const Fr* X = d_evals;  // h = 1: the value is the coefficient
    if (h > 1) {
        Fr* x = ctx->fbuf("idft_X", h * w);
        LSP_HIP(launch_intt(d_evals, ColMap::plain((uint32_t)w), x, w, logh, ctx->twiddle29(logh, true), ctx->stream));
        X = x;
    }
    LSP_HIP(launch_scale_coeffs(X, h, (uint32_t)w, tab, L1, d_out, ctx->stream));
    LSP_HIP(hipStreamSynchronize(ctx->stream));  // `base_scale` is a host temporary
}

// Block `blk` (S = N / 2^b rows, S < h) of the bit-reversed N-row LDE, when a
// proof has more ranks than cosets: the evaluations on the sub-coset
// c H_S, c = shift_c w_N^bitrev_b(blk).  The h coefficients of every column
// fold to S (c'_i = sum_t c_(i + t S) c^(t S), SURVEY 8(e) step 6 without a
// transpose), then one size-S coset NTT of the folded columns, which is
// lde_coeffs_device with the LDE seen as 2^b blocks of S rows.  The fold also
// divides by f = h / S, so the NTT's 1/S twist scale gives the 1/h the
// coefficients (h * c_i, as the inverse leaves them) need.
static void subcoset_lde(lsp_ctx* ctx, const Fr* coef, ColMap map, size_t h, size_t w, uint32_t logN, uint32_t b,
                         uint32_t blk, const Fr* shifts_host, Fr* d_out, const std::string& tag) {
    const size_t S = (size_t)1 << (logN - b), f = h / S;
    LSP_REQUIRE(S < h && f <= 64 && S >= 2, LSP_E_ARG, "sub-coset outside 2 .. h/2 rows");
    const Fr cb = fr_pow_u64(host_two_adic_generator(logN), host_bitrev(blk, b));
    const Fr finv = host_inv_cached(fr_from_u64(f));
    std::vector<Fr> fac(w * f);
    for (size_t c = 0; c < w; ++c) {
        const Fr sigma = fr_pow_u64(fr_mul(shifts_host[c], cb), S);
        Fr x = finv;
        for (size_t t = 0; t < f; ++t) {
            fac[c * f + t] = x;
            x = fr_mul(x, sigma);
        }
    }
    Fr* dfac = ctx->fbuf(tag + "_fac", w * f);
    ctx->h2d_async(tag + "_fac_h", dfac, fac.data(), fac.size() * sizeof(Fr));
    LSP_HIP(launch_to_f29form(dfac, dfac, w * f, ctx->stream));
    Fr* folded = ctx->fbuf(tag + "_fold", S * w);
    LSP_HIP(launch_fold_subcoset(coef, map, h, S, (uint32_t)w, dfac, folded, ctx->stream));
    lde_coeffs_device(ctx, folded, ColMap::plain((uint32_t)w), S, w, b, shifts_host, d_out, blk, 1);
}

// A sharded proof either splits the inverse NTTs by columns (rank g inverts
// the columns bitrev(g) + G k and the coefficients are allgathered; each
// quotient holder inverts its own chunks before their broadcast) or has every
// rank invert every trace column and, after the broadcast of the values, every
// quotient chunk.  The split moves (G - 1) h ceil(w/G) elements into every
// rank and saves (w - ceil(w/G)) h + (q - q/Gq) h elements of inverse NTT (the
// quotient broadcasts carry the same bytes either way); with the communicator
// calibrated (lsp_comm_selftest) the cheaper one is taken -- on the same
// measured numbers on every rank, so the collective schedule stays
// rank-identical.  Uncalibrated (in-process groups, a transport never
// self-tested): the split.  LSP_SHARD_SPLIT_INTT=0/1 forces either (A/B).
// q = 0: the trace's share only.
ExchangePlan exchange_plan(const Comm& comm, size_t h, size_t w, size_t q, uint32_t log_blowup) {
    // read per proof (not cached): tests flip it between proofs in one process
    const char* fe = std::getenv("LSP_SHARD_SPLIT_INTT");
    const int forced = fe && *fe ? (*fe == '0' ? 0 : 1) : -1;
    ExchangePlan p{true, 0, 0, "uncalibrated: split"};
    const size_t G = (size_t)comm.size, cg = (w + G - 1) / G;
    if (comm.ag_gbs > 0 && comm.intt_gelem_s > 0) {
        p.allgather_ms = (double)((G - 1) * h * cg * sizeof(Fr)) / (comm.ag_gbs * 1e9) * 1e3;
        size_t qx = 0;  // quotient chunks a rank inverts beyond its own without the split
        if (q > 0 && G <= ((size_t)1 << log_blowup)) {  // (more ranks than cosets: every rank inverts them anyway)
            const size_t N = h << log_blowup, S = N / G, Q = q * h, Sq = std::min(S, Q), Gq = Q / Sq;
            qx = q - std::max<size_t>(q / Gq, 1);
        }
        p.redundant_ms = (double)((w - std::min(w, cg) + qx) * h) / (comm.intt_gelem_s * 1e9) * 1e3;
        p.split = p.allgather_ms < p.redundant_ms;
        p.reason = p.split ? "measured: allgather cheaper than the redundant inverse"
                           : "measured: redundant inverse cheaper than the allgather";
    }
    if (forced >= 0) {
        p.split = forced == 1;
        p.reason = "forced (LSP_SHARD_SPLIT_INTT)";
    }
    if (G == 1) p.split = false;
    return p;
}

// median wall ms of `reps` runs of f after one warm-up, `before` ahead of each
// run outside the timing (the calibration's barrier)
static double median_ms(lsp_ctx* ctx, const std::function<void()>& f, int reps, const std::function<void()>& before) {
    std::vector<double> t;
    for (int r = 0; r <= reps; ++r) {
        if (before) before();
        LSP_HIP(hipStreamSynchronize(ctx->stream));
        const auto t0 = std::chrono::steady_clock::now();
        f();
        LSP_HIP(hipStreamSynchronize(ctx->stream));
        if (r) t.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

// This GPU's inverse-NTT rate (G elements/s) over an h x w matrix of seeded
// random field elements, h = 2^log_h.  Random operands, not zeros: the chip
// is power-held on MAD-dense work (2.1 against 2.4 GHz), and zero limbs draw
// less power, so an all-zero probe overstates the rate.
// Buffers "calib_intt_x/y" (calibrate_exchange allocates them before its first
// collective; the caller releases them).
double calibrate_intt(lsp_ctx* ctx, uint32_t log_h, size_t w, int reps, const std::function<void()>& before) {
    const size_t h = (size_t)1 << log_h;
    Fr* x = ctx->fbuf("calib_intt_x", h * w);
    Fr* y = ctx->fbuf("calib_intt_y", h * w);
    // h x w values (the raw-column generator: column-major, read here as rows)
    LSP_HIP(launch_gen_raw_perm(0x43414c4942ull /* "CALIB" */, h, (uint32_t)w, 1, 0, x, y, ctx->stream));
    const uint4* tw = ctx->twiddle29(log_h, true);
    // device time between events around a burst of 8 back-to-back inverses
    // (what a proof's phase timer sees of a GPU that is busy): host wall time
    // adds launch and synchronisation latency, and one inverse after an idle
    // gap runs at a clock still ramping up -- 10-13 % slower than the proofs'
    // own phase at 2^20 x 4 (tests/test_gpu_calibration.py)
    constexpr int burst = 8;
    auto inv = [&] { LSP_HIP(launch_intt(x, ColMap::plain((uint32_t)w), y, w, log_h, tw, ctx->stream)); };
    hipEvent_t e0, e1;
    LSP_HIP(hipEventCreate(&e0));
    LSP_HIP(hipEventCreate(&e1));
    std::vector<double> t;
    for (int r = 0; r <= reps; ++r) {
        if (before) before();
        if (!r)
            for (int i = 0; i < burst; ++i) inv();  // warm-up burst
        LSP_HIP(hipEventRecord(e0, ctx->stream));
        for (int i = 0; i < burst; ++i) inv();
        LSP_HIP(hipEventRecord(e1, ctx->stream));
        LSP_HIP(hipEventSynchronize(e1));
        float ms = 0;
        LSP_HIP(hipEventElapsedTime(&ms, e0, e1));
        if (r) t.push_back(ms / burst);
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    std::sort(t.begin(), t.end());
    return (double)(h * w) / (t[t.size() / 2] * 1e-3) / 1e9;
}

void calibrate_exchange(lsp_ctx* ctx, Comm& comm) {
    if (comm.size < 2 || comm.rehearsal()) return;
    hipStream_t st = ctx->stream;
    const size_t G = (size_t)comm.size;
    comm.ag_gbs = comm.intt_gelem_s = 0;
    comm.calib_raw.clear();
    // every rank's k values, in rank order (one small allgather)
    double* ds = (double*)ctx->buf("calib_ds", 4 * sizeof(double));
    double* dr = (double*)ctx->buf("calib_dr", 4 * sizeof(double) * G);
    auto gather = [&](const std::vector<double>& mine) {
        const size_t k = mine.size();
        LSP_HIP(hipMemcpyAsync(ds, mine.data(), k * sizeof(double), hipMemcpyHostToDevice, st));
        comm.allgather(ctx, ds, dr, k * sizeof(double), "calibration");
        std::vector<double> all(k * G);
        LSP_HIP(hipMemcpyAsync(all.data(), dr, all.size() * sizeof(double), hipMemcpyDeviceToHost, st));
        LSP_HIP(hipStreamSynchronize(st));
        return all;
    };
    // a barrier ahead of every timed rep, so no rank's time includes waiting for a late peer
    auto barrier = [&] {
        LSP_HIP(hipMemsetAsync(ds, 0, sizeof(double), st));
        comm.allgather(ctx, ds, dr, sizeof(double), "calibration barrier");
        LSP_HIP(hipStreamSynchronize(st));
    };
    // Every buffer first: a rank that cannot allocate must not
    // leave its peers blocked in a collective it never joins.  The ranks agree
    // on success with one allgather; on any failure all of them skip the
    // probes and stay uncalibrated (the split exchange), consistently.
    const uint32_t logh = 20;
    const size_t h = (size_t)1 << logh, w = 8;
    const size_t big = (size_t)256 << 20, share_big = std::max<size_t>(big / G / 256, 1) * 256;
    double ok = 1;
    try {
        ctx->buf("calib_s", share_big);
        ctx->buf("calib_r", share_big * G);
        ctx->fbuf("calib_intt_x", h * w);
        ctx->fbuf("calib_intt_y", h * w);
        ctx->twiddle29(logh, true);
    } catch (const LspError&) {
        ok = 0;
        (void)hipGetLastError();
    }
    const std::vector<double> oks = gather({ok});
    if (*std::min_element(oks.begin(), oks.end()) == 0) {
        comm.calib_status = "skipped: a rank could not allocate the probe buffers";
        ctx->release("calib_");
        return;
    }
    // the allgather: a 4 MiB probe first; only a transport that is not clearly
    // below the break-even region (>= 20 GB/s on every rank) gets the 256 MiB one
    auto probe = [&](size_t total) {
        const size_t share = std::max<size_t>(total / G / 256, 1) * 256;
        char* s = (char*)ctx->buf("calib_s", share_big);
        char* r = (char*)ctx->buf("calib_r", share_big * G);
        LSP_HIP(hipMemsetAsync(s, comm.rank & 0xff, share, st));
        const double ms = median_ms(ctx, [&] { comm.allgather(ctx, s, r, share, "calibration"); }, 3, barrier);
        comm.ag_probe_bytes = share * G;
        return (double)((G - 1) * share) / (ms * 1e-3) / 1e9;
    };
    const double small = probe((size_t)4 << 20);
    const std::vector<double> smalls = gather({small});
    const bool go_big = *std::min_element(smalls.begin(), smalls.end()) >= 20;  // the same on every rank
    const double large = go_big ? probe(big) : 0.0;
    if (!go_big) comm.ag_probe_bytes = std::max<size_t>(((size_t)4 << 20) / G / 256, 1) * 256 * G;
    // the inverse NTT the split distributes: 8 columns of 2^20 of random field elements
    const double intt = calibrate_intt(ctx, logh, w, 3, barrier);
    comm.calib_raw = gather({small, large, intt});  // 3 per rank, rank order (lsp_comm_calibration)
    double gbs = 1e300, rate = 1e300;
    for (size_t r = 0; r < G; ++r) {
        gbs = std::min(gbs, go_big ? comm.calib_raw[3 * r + 1] : comm.calib_raw[3 * r]);
        rate = std::min(rate, comm.calib_raw[3 * r + 2]);
    }
    comm.ag_gbs = gbs;
    comm.intt_gelem_s = rate;
    comm.calib_status = go_big ? "calibrated (4 MiB and 256 MiB allgather probes, random-data inverse NTT)"
                               : "calibrated (4 MiB allgather probe below 20 GB/s, random-data inverse NTT)";
    ctx->release("calib_");
}

QuotientExchange quotient_exchange(const Comm& comm, size_t h, size_t q, uint32_t log_blowup) {
    QuotientExchange x{0, 0, 0};
    const size_t G = (size_t)comm.size;
    if (G < 2 || q == 0) return x;
    const size_t N = h << log_blowup, S = N / G, Q = q * h, Sq = std::min(S, Q);
    x.bcasts = Q / Sq;
    x.bytes_each = Sq * sizeof(Fr);
    if (comm.ag_gbs > 0) x.model_ms = (double)(x.bcasts * x.bytes_each) / (comm.ag_gbs * 1e9) * 1e3;
    return x;
}

// ------------------------------------------------------------- Merkle
// MerkleTreeMmcs::commit of `m` into `layers` (2*height - 1 digests, leaves
// first).  Wide levels run on the GPU; once a layer has at most
// host_tree_top digests the remaining levels are a few dozen permutations on
// the critical path, and the host (a ~30 ns multiply against ~350 ns for one
// wave's multiply chain) finishes them with a small thread pool.  Trees of
// at most host_tree_top single-matrix rows are hashed on the host entirely.
// The host layers go back to the device (openings gather from device memory)
// from a pinned staging buffer, without waiting: the next use of the buffer
// comes after a later synchronisation of the same stream.
// LSP_TIME_TOPS=1: host-side timing of the tree tops (diagnostic), printed at exit
struct TopTimes {
    bool on = std::getenv("LSP_TIME_TOPS") != nullptr;
    double sync_us = 0, levels_us = 0, first_us = 0;
    size_t n = 0;
    // per tree (the last ones are printed): host time since the previous tree's
    // return, launch issue, sleep until ev_near, spin until ev_top, host levels
    struct Rec { size_t height; double since_prev, launch, near, spin, levels; };
    std::vector<Rec> recs;
    std::chrono::steady_clock::time_point last_exit{};
    ~TopTimes() {
        if (on && n) {
            std::fprintf(stderr, "[tree tops] %zu trees: wait-for-GPU %.1f us, host levels %.1f us (first level %.1f us) per tree\n",
                         n, sync_us / n, levels_us / n, first_us / n);
            const size_t k = recs.size() < 16 ? 0 : recs.size() - 16;
            for (size_t i = k; i < recs.size(); ++i)
                std::fprintf(stderr, "[tree] height %9zu  since-prev %7.1f  launch %6.1f  near %8.1f  spin %7.1f  levels %6.1f us\n",
                             recs[i].height, recs[i].since_prev, recs[i].launch, recs[i].near, recs[i].spin, recs[i].levels);
        }
    }
};
static TopTimes g_top_times;

// Proofs running at once in this process (several contexts in flight, or the
// ranks of an in-process group).  A lone proof hands its trees to the host
// pool from host_tree_top digests; concurrent proofs share the host's cores,
// so there the host takes over only from 256 digests (bench, same box:
// 1024 vs 256 = 67.6 vs 68.3 ms alone, 62.3 vs 60.0 ms per proof with three in flight).
static std::atomic<int> g_active_proofs{0};
struct ActiveProof {
    ActiveProof() { g_active_proofs.fetch_add(1, std::memory_order_relaxed); }
    ~ActiveProof() { g_active_proofs.fetch_sub(1, std::memory_order_relaxed); }
};
constexpr size_t SHARED_HOST_TREE_TOP = 256;

// out[i] = compress(in[2i], in[2i+1]) for i < half on the host pool
static void host_compress_level(lsp_ctx* ctx, const Fr* in, Fr* out, size_t half) {
    HostPool& pool = ctx->host_pool();
    if (half <= pool.size())  // one permutation per thread: the scalar path's latency is lower
        pool.parallel_for(half, [&](size_t i) { out[i] = ctx->p2.compress(in[2 * i], in[2 * i + 1]); });
    else {  // 8 or 16 at a time (AVX-512 IFMA when the CPU has it)
        const size_t blk = half >= 16 * pool.size() ? 16 : 8;
        pool.parallel_for((half + blk - 1) / blk, [&](size_t b) {
            ctx->p2.compress_range(in, out, blk * b, std::min(half, blk * b + blk));
        });
    }
}

// Round 3's host levels (LSP_HOST_LEVELS=r3, for same-box A/B): level by
// level while a level has more than 16 digests per thread, then subtrees of 16.
// Wide levels go level by level through the pool (work shared dynamically).
// Once a level holds at most 16 digests per pool thread, the rest of the tree
// is P = n / 16 subtrees of 16 digests, one task each (no barrier between their
// levels: a parallel_for costs ~5 us, more than an 8-lane IFMA batch), and the
// levels above the P subtree roots run on this thread.  The workers are awake
// then (they just ran the level below).  LSP_HOST_SUBTREE=0: level by level.
static size_t host_levels_r3(lsp_ctx* ctx, Fr* host, size_t first,
                             std::chrono::steady_clock::time_point* t_first) {
    static const bool subtrees = [] {
        const char* e = std::getenv("LSP_HOST_SUBTREE");
        return !(e && *e == '0');
    }();
    constexpr size_t SUB = 16;  // digests per subtree task
    HostPool& pool = ctx->host_pool();
    size_t lo = 0, n = first, end = first;
    while (n > 1 && (!subtrees || n > SUB * pool.size())) {
        host_compress_level(ctx, host + lo, host + end, n / 2);
        if (lo == 0 && t_first) *t_first = std::chrono::steady_clock::now();
        lo = end;
        end += n / 2;
        n /= 2;
    }
    if (n <= 1) return end;
    // n (a power of two, <= SUB * threads) digests at host[lo, lo + n): level
    // j >= 1 above them holds n >> j digests at off[j]
    size_t off[64];
    uint32_t nl = 0;
    off[0] = lo;
    for (size_t c = n / 2; c >= 1; c /= 2) {
        off[++nl] = end;
        end += c;
    }
    auto level_part = [&](uint32_t j, size_t i0, size_t cnt) {  // level j, digests [i0, i0 + cnt)
        if (cnt == 1)
            host[off[j] + i0] = ctx->p2.compress(host[off[j - 1] + 2 * i0], host[off[j - 1] + 2 * i0 + 1]);
        else
            ctx->p2.compress_range(host + off[j - 1], host + off[j], i0, i0 + cnt);
    };
    const uint32_t sl = n >= SUB ? log2_exact(SUB) : 0;  // levels inside a subtree task
    if (sl)
        pool.parallel_for(n / SUB, [&](size_t p) {
            for (uint32_t j = 1; j <= sl; ++j) level_part(j, p * (SUB >> j), SUB >> j);
        });
    for (uint32_t j = sl + 1; j <= nl; ++j) level_part(j, 0, n >> j);  // above the subtree roots
    if (lo == 0 && t_first) *t_first = std::chrono::steady_clock::now();
    return end;
}

// The levels above `first` digests host[0, first): each level is appended
// after the one below it; returns the end of the layers (the root is
// host[end - 1]).  *t_first (if given) is set after the first level.
// pairs (optional): the `first` digests are made first, as the 2-element
// leaves compress(pairs[2i], pairs[2i+1]) of a FRI round (A4/A5), inside the
// same tasks.
// The tree splits into P = (pool threads, a power of two) subtrees of
// first / P digests, one task each: a task hashes its leaves and every level
// of its subtree with no barrier in between (a parallel_for costs ~5 us, as
// much as an 8-lane IFMA batch, and the levels below 16 digests per thread
// used to take one each), and the log2 P levels above the subtree roots run on
// this thread.  Each task keeps >= 16 digests (fewer threads for small
// trees).  LSP_HOST_SUBTREE=0: level by level, one parallel_for each.
static size_t host_levels(lsp_ctx* ctx, Fr* host, size_t first,
                          std::chrono::steady_clock::time_point* t_first = nullptr, const Fr* pairs = nullptr) {
    static const bool subtrees = [] {
        const char* e = std::getenv("LSP_HOST_SUBTREE");
        return !(e && *e == '0');
    }();
    HostPool& pool = ctx->host_pool();
    if (const char* e = std::getenv("LSP_HOST_LEVELS"); e && e[0] == 'r') {  // A/B: round 3's levels
        if (pairs) host_compress_level(ctx, pairs, host, first);
        return host_levels_r3(ctx, host, first, t_first);
    }
    if (first <= 1) {
        if (pairs && first == 1) host[0] = ctx->p2.compress(pairs[0], pairs[1]);
        if (t_first) *t_first = std::chrono::steady_clock::now();
        return first;
    }
    // level j >= 0 holds first >> j digests at off[j]
    size_t off[64];
    uint32_t nl = 0;
    off[0] = 0;
    size_t end = first;
    for (size_t c = first / 2; c >= 1; c /= 2) {
        off[++nl] = end;
        end += c;
    }
    auto level_part = [&](uint32_t j, size_t i0, size_t cnt) {  // level j, digests [i0, i0 + cnt)
        if (cnt == 1)
            host[off[j] + i0] = ctx->p2.compress(host[off[j - 1] + 2 * i0], host[off[j - 1] + 2 * i0 + 1]);
        else
            ctx->p2.compress_range(host + off[j - 1], host + off[j], i0, i0 + cnt);
    };
    auto leaf_part = [&](size_t i0, size_t cnt) {
        if (cnt == 1)
            host[i0] = ctx->p2.compress(pairs[2 * i0], pairs[2 * i0 + 1]);
        else
            ctx->p2.compress_range(pairs, host, i0, i0 + cnt);
    };
    if (!subtrees) {
        if (pairs) host_compress_level(ctx, pairs, host, first);
        for (uint32_t j = 1; j <= nl; ++j) {
            host_compress_level(ctx, host + off[j - 1], host + off[j], first >> j);
            if (j == 1 && t_first) *t_first = std::chrono::steady_clock::now();
        }
        return end;
    }
    size_t P = 1;
    while (2 * P <= pool.size() && first / (2 * P) >= 16) P *= 2;
    const size_t per = first / P;
    const uint32_t sl = log2_exact(per);  // levels inside a task
    auto task = [&](size_t p) {
        if (pairs) leaf_part(p * per, per);
        for (uint32_t j = 1; j <= sl; ++j) level_part(j, p * (per >> j), per >> j);
    };
    if (P > 1)
        pool.parallel_for(P, task);
    else
        task(0);
    if (t_first) *t_first = std::chrono::steady_clock::now();
    for (uint32_t j = sl + 1; j <= nl; ++j) level_part(j, 0, first >> j);  // above the task roots
    return end;
}

// the pinned buffer of a tree's host layers: one per tree while uploads are
// deferred (each must stay intact until flush_top_uploads), else one shared
static std::string top_buf_name(lsp_ctx* ctx) {
    return ctx->defer_top_uploads ? "merkle_top" + std::to_string(ctx->top_uploads.size()) : std::string("merkle_top");
}

// issue the deferred tree-top uploads on the context's stream
static void flush_top_uploads(lsp_ctx* ctx) {
    for (const auto& u : ctx->top_uploads)
        LSP_HIP(hipMemcpyAsync(u.dst, u.src, u.bytes, hipMemcpyHostToDevice, ctx->stream));
    ctx->top_uploads.clear();
}

// defers the uploads for one proof; the destructor drops any left (an error path)
struct DeferTopUploads {
    lsp_ctx* ctx;
    explicit DeferTopUploads(lsp_ctx* c) : ctx(c) {
        ctx->top_uploads.clear();
        ctx->defer_top_uploads = std::getenv("LSP_NO_DEFER_TOPS") == nullptr;
    }
    ~DeferTopUploads() {
        ctx->defer_top_uploads = false;
        ctx->top_uploads.clear();
    }
};

// LSP_TOP_ZEROCOPY=0: the last GPU level goes to HBM and a copy brings it to the host
static bool zerocopy_top() {
    static const bool on = [] {
        const char* e = std::getenv("LSP_TOP_ZEROCOPY");
        return !(e && *e == '0');
    }();
    return on;
}

// levels above this many digests fill the chip; the ones below run one wave per
// SIMD or fewer (per-level rates)
constexpr size_t WIDE_LEVEL_STOP = (size_t)1 << 16;

// The host pool starts spinning when a tree's GPU levels are down to this many
// digests (ev_warm), not only for the last two levels (ev_near): after a GPU
// phase of milliseconds the pool's cores, asleep meanwhile, ran the tree top's
// first parallel_for 20-75 us slower than cores kept busy, unless they had been
// spinning for about a millisecond (LSP_TIME_TOPS per tree: 2^16 and 2^18 still
// left the 4M-leaf trees slow, 2^20 -- 1.5-2.7 ms ahead -- made every tree top
// as fast as the narrow trees').  Read per call; LSP_TOP_WARM=0: off.  By
// default only while this proof has the host to itself: with several proofs in
// flight in the process or several ranks on the host (LOCAL_WORLD_SIZE > 1) the
// pools' spinning competed with the other proofs' host work (eight ranks
// sharing one GPU and 16 CPUs: 19 % slower), for nothing the GPU waits on.
static size_t top_warm_nodes(const lsp_ctx* ctx) {
    if (const char* e = std::getenv("LSP_TOP_WARM")) return (size_t)std::strtoull(e, nullptr, 10);
    static const bool shared_host = [] {
        const char* e = std::getenv("LOCAL_WORLD_SIZE");
        return e && std::strtol(e, nullptr, 10) > 1;
    }();
    if (shared_host || ctx->comm || g_active_proofs.load(std::memory_order_relaxed) > 1) return 0;
    return (size_t)1 << 20;
}
constexpr unsigned TOP_WARM_SPIN_US = 5000;  // bound on the pool's spin after ev_warm

Fr commit_device(lsp_ctx* ctx, const MatList& m, size_t height, Fr* layers, const FoldSpec* fold,
                 const std::function<void(hipEvent_t)>* side) {
    hipStream_t st = ctx->stream;
    using clk = std::chrono::steady_clock;
    const auto tt0 = clk::now();
    auto t_launched = tt0, t_near = tt0;
    size_t top = ctx->host_tree_top;
    if (g_active_proofs.load(std::memory_order_relaxed) > 1) top = std::min(top, SHARED_HOST_TREE_TOP);
    if (const char* e = std::getenv("LSP_HOST_TREE_TOP")) top = std::strtoull(e, nullptr, 10);
    HostPool& pool = ctx->host_pool();
    size_t off = 0, len = height;
    if (fold && height <= top && height > 1) {
        // a short vector: materialise the fold, then the host path below hashes it
        LSP_HIP(launch_fri_fold(fold->v, 2 * height, fold->half, fold->half_beta, fold->tab, fold->L1, fold->vout, st,
                                fold->i0, (int)fold->logm));
        fold = nullptr;
    }
    const bool leaves_on_host = height <= top && m.n == 1 && height > 1;
    bool gpu_level_on_host = false;  // the last GPU level was written into `host` directly
    Fr* host;  // host layers, starting at device offset `off` (pinned)
    if (leaves_on_host) {
        const size_t w = m.width[0];
        host = (Fr*)ctx->hbuf(top_buf_name(ctx), (2 * height - 1 + height * w) * sizeof(Fr));
        Fr* rows = host + 2 * height - 1;
        LSP_HIP(hipMemcpyAsync(rows, m.ptr[0], height * w * sizeof(Fr), hipMemcpyDeviceToHost, st));
        if (side) {  // nothing left on the GPU for this tree
            LSP_HIP(hipEventRecord(ctx->ev_wide, st));
            (*side)(ctx->ev_wide);
        }
        LSP_HIP(hipStreamSynchronize(st));
        pool.parallel_for((height + 7) / 8, [&](size_t b) {
            ctx->p2.hash_range(rows, w, host, 8 * b, std::min(height, 8 * b + 8));
        });
    } else {
        if (fold)
            LSP_HIP(launch_fold_hash(*fold, height, layers, ctx->rc29_dev, ctx->p2.L, st));
        else
            LSP_HIP(launch_hash_rows(m, height, layers, ctx->rc29_dev, ctx->p2.L, st));
        if (top == 0) {
            LSP_HIP(launch_merkle_tree(layers, height, ctx->rc29_dev, ctx->p2.L, st));
            if (side) {
                LSP_HIP(hipEventRecord(ctx->ev_wide, st));
                (*side)(ctx->ev_wide);
            }
            return d2h_fr(ctx, layers + 2 * height - 2);
        }
        if (!ctx->ev_near) {
            LSP_HIP(hipEventCreateWithFlags(&ctx->ev_near, hipEventDisableTiming));
            LSP_HIP(hipEventCreateWithFlags(&ctx->ev_top, hipEventDisableTiming));
            LSP_HIP(hipEventCreateWithFlags(&ctx->ev_warm, hipEventDisableTiming));
        }
        // the wide levels; the side work's / the host pool's event; the narrow ones
        // down to 4 top; an event; the last two (~100 us) and the download
        const size_t warm = top_warm_nodes(ctx);
        // stops (largest first) after which an event goes on the stream
        struct Stop {
            size_t nodes;
            hipEvent_t ev;
        } stops[2];
        int nstops = 0;
        if (warm) stops[nstops++] = {std::max(4 * top, warm), ctx->ev_warm};
        if (side) stops[nstops++] = {std::max(4 * top, WIDE_LEVEL_STOP), ctx->ev_wide};
        if (nstops == 2 && stops[1].nodes > stops[0].nodes) std::swap(stops[0], stops[1]);
        size_t off1 = 0, len1 = height;
        for (int k = 0; k < nstops; ++k) {
            size_t o = 0, l = len1;
            LSP_HIP(launch_merkle_levels(layers + off1, len1, stops[k].nodes, ctx->rc29_dev, ctx->p2.L, &o, &l, st));
            LSP_HIP(hipEventRecord(stops[k].ev, st));
            off1 += o;
            len1 = l;
        }
        {
            size_t o = 0, l = len1;
            LSP_HIP(launch_merkle_levels(layers + off1, len1, 4 * top, ctx->rc29_dev, ctx->p2.L, &o, &l, st));
            off1 += o;
            len1 = l;
        }
        LSP_HIP(hipEventRecord(ctx->ev_near, st));
        size_t off2 = 0, len2 = len1;
        if (zerocopy_top())
            LSP_HIP(launch_merkle_levels(layers + off1, len1, 2 * top, ctx->rc29_dev, ctx->p2.L, &off2, &len2, st));
        if (zerocopy_top() && len2 > top) {
            // down to 2 top digests in HBM; the last GPU level writes its `top`
            // digests straight into the pinned host buffer (no copy kernel on the
            // critical path); the upload below takes them back to HBM
            off = off1 + off2;
            len = len2 / 2;
            // fine-grained (coherent) pinned memory: the kernel's stores bypass the
            // GPU caches, so they are in host memory when the kernel completes
            host = (Fr*)ctx->hbuf(top_buf_name(ctx) + "c", (2 * len - 1) * sizeof(Fr), hipHostMallocCoherent);
            LSP_HIP(launch_merkle_level(layers + off, host, len, ctx->rc29_dev, ctx->p2.L, st));
            off += len2;
            gpu_level_on_host = true;
        } else if (zerocopy_top()) {  // no GPU level left above `top` digests: copy them
            off = off1 + off2;
            len = len2;
            host = (Fr*)ctx->hbuf(top_buf_name(ctx), (2 * len - 1) * sizeof(Fr));
            LSP_HIP(hipMemcpyAsync(host, layers + off, len * sizeof(Fr), hipMemcpyDeviceToHost, st));
        } else {
            LSP_HIP(launch_merkle_levels(layers + off1, len1, top, ctx->rc29_dev, ctx->p2.L, &off, &len, st));
            off += off1;
            host = (Fr*)ctx->hbuf(top_buf_name(ctx), (2 * len - 1) * sizeof(Fr));
            LSP_HIP(hipMemcpyAsync(host, layers + off, len * sizeof(Fr), hipMemcpyDeviceToHost, st));
        }
        LSP_HIP(hipEventRecord(ctx->ev_top, st));
        if (side) (*side)(ctx->ev_wide);
        t_launched = clk::now();
        // sleep through the wide levels, then spin (with the pool awake) for the last ones
        resolve_timings(ctx);  // the previous proof's phase events, meanwhile
        hipError_t q;
        if (warm) {
            LSP_HIP(hipEventSynchronize(ctx->ev_warm));
            pool.wake(TOP_WARM_SPIN_US);
            while ((q = hipEventQuery(ctx->ev_near)) == hipErrorNotReady) {
#if defined(__x86_64__)
                __builtin_ia32_pause();
#endif
            }
            LSP_HIP(q);
            t_near = clk::now();
        } else {
            LSP_HIP(hipEventSynchronize(ctx->ev_near));
            t_near = clk::now();
            pool.wake();
        }
        while ((q = hipEventQuery(ctx->ev_top)) == hipErrorNotReady) {
#if defined(__x86_64__)
            __builtin_ia32_pause();
#endif
        }
        LSP_HIP(q);
    }
    const auto tt1 = clk::now();
    auto tt2 = tt1;
    const size_t first = len;  // the part already on the device (unless hashed here)
    const size_t end = host_levels(ctx, host, first, &tt2);
    if (g_top_times.on) {
        const auto tt3 = clk::now();
        g_top_times.n++;
        g_top_times.sync_us += std::chrono::duration<double, std::micro>(tt1 - tt0).count();
        g_top_times.levels_us += std::chrono::duration<double, std::micro>(tt3 - tt1).count();
        g_top_times.first_us += std::chrono::duration<double, std::micro>(tt2 - tt1).count();
        auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        g_top_times.recs.push_back({height, g_top_times.last_exit == clk::time_point{} ? 0.0 : us(g_top_times.last_exit, tt0),
                                    us(tt0, t_launched), us(t_launched, t_near), us(t_near, tt1), us(tt1, tt3)});
        g_top_times.last_exit = clk::now();
    }
    // digests that exist only on the host start here
    const size_t skip = leaves_on_host || gpu_level_on_host ? 0 : first;
    if (end > skip) {
        if (ctx->defer_top_uploads)
            ctx->top_uploads.push_back({layers + off + skip, host + skip, (end - skip) * sizeof(Fr)});
        else
            LSP_HIP(hipMemcpyAsync(layers + off + skip, host + skip, (end - skip) * sizeof(Fr), hipMemcpyHostToDevice, st));
    }
    return host[end - 1];
}

static MatList one_mat(const Fr* p, uint32_t w) {
    MatList m{};
    m.ptr[0] = p;
    m.width[0] = w;
    m.n = 1;
    return m;
}

// --------------------------------------------------------------- grind
// GrindingChallenger::grind(bits) on the device: the smallest witness w >= 0
// with sample_bits(bits) == 0 after observe(w) (U8).  The sponge over the
// challenger's input buffer is absorbed on the host up to the block that
// will hold w; the device runs the last permutation for 2^22 candidates per
// launch.  The winner is re-checked on the host transcript.
uint64_t grind_device(lsp_ctx* ctx, Challenger& ch, uint32_t bits) {
    if (bits == 0) {
        LSP_REQUIRE(ch.check_witness(0, 0), LSP_E_STATE, "grind(0) must accept w = 0");
        return 0;
    }
    const std::vector<Fr>& in = ch.in;  // observe(w) clears the output buffer and appends w
    Fr s0 = fr_zero(), s1 = fr_zero(), s2 = fr_zero();
    size_t k = 0;
    while (k + 2 <= in.size()) {
        s0 = in[k];
        s1 = in[k + 1];
        ctx->p2.permute(s0, s1, s2);
        k += 2;
    }
    uint32_t wlane;
    Fr pre[3];
    if (k < in.size()) {  // odd prefix: [last, w] form the final block
        pre[0] = in[k];
        pre[1] = s1;
        pre[2] = s2;
        wlane = 1;
    } else {  // even prefix: w alone in lane 0, lane 1 keeps the previous state
        pre[0] = s0;
        pre[1] = s1;
        pre[2] = s2;
        wlane = 0;
    }
    unsigned long long* best = (unsigned long long*)ctx->buf("grind_best", sizeof(unsigned long long));
    const uint64_t batch = 1ull << 22;
    for (uint64_t base = 0;; base += batch) {
        LSP_HIP(hipMemsetAsync(best, 0xff, sizeof(unsigned long long), ctx->stream));
        LSP_HIP(launch_grind(pre, wlane, base, batch, bits, ch.mont_bits, ctx->rc29_dev, ctx->p2.L, best, ctx->stream));
        unsigned long long got = 0;
        LSP_HIP(hipMemcpyAsync(&got, best, sizeof(got), hipMemcpyDeviceToHost, ctx->stream));
        LSP_HIP(hipStreamSynchronize(ctx->stream));
        if (got != ~0ull) {
            LSP_REQUIRE(ch.check_witness(bits, got), LSP_E_STATE, "device grind witness rejected by the transcript");
            return got;
        }
        LSP_REQUIRE(base < (1ull << 50), LSP_E_STATE, "grinding did not terminate");
    }
}

// ------------------------------------------------------------- prove
// Root of a Merkle tree whose 2^b bottom subtrees live on the 2^b ranks
// (rank r's subtree root = `local`, leaves r*S .. (r+1)*S - 1).  `top` gets
// the b + 1 host layers above the subtrees (top[0] = the rank roots).
static Fr shard_root(lsp_ctx* ctx, Comm& comm, const Fr& local, std::vector<std::vector<Fr>>& top, const char* tag) {
    if (comm.size == 1) {
        top.assign(1, std::vector<Fr>(1, local));
        return local;
    }
    top.assign(1, comm.allgather_fr(ctx, &local, 1, tag));
    while (top.back().size() > 1) {
        const std::vector<Fr>& lo = top.back();
        std::vector<Fr> up(lo.size() / 2);
        for (size_t i = 0; i < up.size(); ++i) up[i] = ctx->p2.compress(lo[2 * i], lo[2 * i + 1]);
        top.push_back(std::move(up));
    }
    return top.back()[0];
}

// p3_uni_stark::prove (bin/src/main.rs:80-86) as one rank of a G-rank
// proof; G = 1 is the single-GPU prover.  Rank g owns the
// LDE rows [g S, (g+1) S), S = N / G: whole cosets of the bit-reversed LDE
// (G <= blowup), hence a whole subtree of every input Merkle tree, the
// quotient points whose rows it holds, and a contiguous slice of every FRI
// vector.  Exchanges: subtree roots, the quotient chunks (one allgather),
// the opened values (each computed on one rank's first coset, allgathered), the
// FRI vector once a slice is shorter than FRI_SHARD_MIN, and the query
// openings.  The transcript runs on every rank with identical inputs.
lsp_proof* prove_shard(lsp_ctx* ctx, Comm& comm, const Fr* d_trace, size_t h, size_t w, const Air& air,
                       const Fr* pub, size_t npub) {
    LSP_REQUIRE(npub >= 2, LSP_E_ARG, "public values must hold [alpha, delta]");
    LSP_REQUIRE(air.max_col < w, LSP_E_ARG, "AIR column id outside the trace width");
    const auto t_entry = std::chrono::steady_clock::now();
    const ActiveProof active;
    const DeferTopUploads defer(ctx);
    comm.begin_log(ctx);
    const uint32_t log_h = log2_exact(h);
    LSP_REQUIRE(h >= 2, LSP_E_SIZE, "trace needs at least 2 rows");
    const uint32_t lb = ctx->log_blowup;
    const uint32_t log_q = air.log_quotient_degree(ctx->public_degree);
    LSP_REQUIRE(log_q <= lb, LSP_E_ARG, "quotient degree exceeds the blowup");
    const size_t q = (size_t)1 << log_q;
    const uint32_t logN = log_h + lb, logQ = log_h + log_q;
    const size_t N = (size_t)1 << logN, Q = (size_t)1 << logQ;
    LSP_REQUIRE(logN <= 40, LSP_E_SIZE, "trace too large");
    const uint32_t G = (uint32_t)comm.size, g = (uint32_t)comm.rank;
    const uint32_t b = log2_exact(G);
    LSP_REQUIRE(b <= lb + 6, LSP_E_ARG, "a proof shards over at most 2^(log_blowup + 6) ranks");
    LSP_REQUIRE(b < logN, LSP_E_SIZE, "more ranks than LDE rows / 2");
    const uint32_t logS = logN - b;
    const size_t S = N >> b, row0 = (size_t)g * S;
    // G <= 2^lb: rank g owns the whole cosets [k0, k0 + nk).  G > 2^lb (sub): a
    // sub-coset of S < h rows, folded from the coefficients (subcoset_lde)
    const bool sub = b > lb;
    const uint32_t nk = sub ? 1u : 1u << (lb - b), k0 = sub ? g : g * nk;
    hipStream_t st = ctx->stream;
    const Fr GEN = host_generator();
    const Fr one = fr_one();
    PhaseTimer T(ctx);
    auto* proof = new lsp_proof();
    // the logical operations of p3_uni_stark::prove with their dims, worded as
    // the reference's tracing spans (bench.log:19-64); batched launches below
    // are logged per reference call (one quotient chunk, one opened matrix)
    ctx->spans.clear();
    auto span = [&](const char* name, size_t rows_w, size_t height, int added_bits) {
        char s[160];
        if (added_bits >= 0)
            std::snprintf(s, sizeof s, "%s dims: %zux%zu | added_bits: %d", name, rows_w, height, added_bits);
        else
            std::snprintf(s, sizeof s, "%s dims: %zux%zu", name, rows_w, height);
        ctx->spans.emplace_back(s);
    };
    proof->log_h = log_h;
    proof->log_q = log_q;
    proof->w = (uint32_t)w;
    proof->rehearsal = comm.rehearsal();
    try {
        T.begin("prove");
        // ---- commit to trace data
        T.begin("commit to trace data");
        Fr* lde = ctx->fbuf("t_lde", S * w);
        std::vector<Fr> shifts(std::max(w, q), GEN);
        T.begin("coset_lde_batch");
        span("coset_lde_batch", w, h, (int)lb);
        const bool split = G > 1 && exchange_plan(comm, h, w, q, lb).split;
        const Fr* tcoef = nullptr;  // h * coefficients of the trace (split or sub), read through tmap
        ColMap tmap;
        if (split) {
            // rank g inverts the columns bitrev(g) + G k (k < cg; columns past w
            // are zero padding), the ranks allgather the h x cg coefficient
            // blocks, and each transforms its own cosets from them
            const uint32_t cg = (uint32_t)((w + G - 1) / G);
            Fr* xl = ctx->fbuf("t_coef_local", h * cg);
            Fr* coef = ctx->fbuf("t_coef", h * cg * G);
            ColMap m = ColMap::plain((uint32_t)w);
            m.c0 = (uint32_t)host_bitrev(g, b);
            m.cstep = G;
            T.begin("trace inverse NTT");  // this rank's cg columns (tests/test_gpu_calibration.py)
            LSP_HIP(launch_intt(d_trace, m, xl, cg, log_h, ctx->twiddle29(log_h, true), st));
            T.end("trace inverse NTT");
            comm.allgather(ctx, xl, coef, h * cg * sizeof(Fr), "trace coefficients");
            tcoef = coef;
            tmap = ColMap::blocked(b, cg);
        } else if (sub) {  // every rank inverts every column (LSP_SHARD_SPLIT_INTT=0)
            Fr* coef = ctx->fbuf("t_coef", h * w);
            LSP_HIP(launch_intt(d_trace, ColMap::plain((uint32_t)w), coef, w, log_h, ctx->twiddle29(log_h, true), st));
            tcoef = coef;
            tmap = ColMap::plain((uint32_t)w);
        }
        if (sub)
            subcoset_lde(ctx, tcoef, tmap, h, w, logN, b, g, shifts.data(), lde, "t_sub");
        else if (split)
            lde_coeffs_device(ctx, tcoef, tmap, h, w, lb, shifts.data(), lde, k0, nk);
        else
            lde_device(ctx, d_trace, h, w, lb, shifts.data(), lde, k0, nk);
        const auto t_lde_issued = std::chrono::steady_clock::now();
        T.end("coset_lde_batch");
        // ---- quotient set-up (nothing here depends on alpha).  Point i reads LDE
        // rows bitrev_Q(i) and bitrev_Q(i + q): the ranks holding the first Q rows
        // (Gq of them) each own the points
        // i = bitrev(g) mod Gq, which are whole chunks j = i mod q (Gq <= q).
        const size_t Sq = std::min(S, Q), Gq = Q / Sq, cpr = q / Gq;
        const uint32_t logGq = log2_exact(Gq);
        uint32_t L1Q;
        const Fr* tabQ = pow_table(ctx, "tabQ", host_two_adic_generator(logQ), logQ, L1Q);
        const Fr wh = host_two_adic_generator(log_h);
        const Fr wh_inv = host_inv_cached(wh);
        // G = 1: the h x q chunk matrix.  G > 1: ranks g < Gq evaluate points
        // into their slot of the exchange buffer (split: into a local buffer,
        // whose inverse NTT goes to the slot)
        // sub: a chunk spreads over Gq / q ranks, so the holders broadcast values
        // and every rank inverts the assembled h x q matrix
        const bool qsplit = split && !sub;
        Fr* qv = G == 1 || !qsplit ? ctx->fbuf("q_values", Q) : nullptr;
        Fr* stage = G == 1 ? nullptr : ctx->fbuf("q_stage", Sq * Gq);
        Fr* qloc = G == 1 ? qv : (g < Gq ? (qsplit ? ctx->fbuf("q_vals_local", Sq) : stage + (size_t)g * Sq) : nullptr);
        // point i + q (the next trace row) of this rank's points i = i0 + Gq m:
        // on this rank when Gq <= q; else all on the rank with residue
        // (i0 + q) mod Gq, whose LDE rows this rank computes itself
        const Fr* lde_next = nullptr;
        uint64_t row0_next = 0;
        if (sub && row0 < Q) {
            const uint32_t gn = (uint32_t)host_bitrev((host_bitrev(g, logGq) + q) & (Gq - 1), logGq);
            if (gn != g) {
                Fr* nl = ctx->fbuf("t_lde_next", S * w);
                subcoset_lde(ctx, tcoef, tmap, h, w, logN, b, gn, shifts.data(), nl, "t_next");
                lde_next = nl;
                row0_next = (uint64_t)gn * S;
            }
        }
        std::vector<Fr> zh(q), izh(q);
        QuotientArgs qa;  // alpha set once sampled
        if (row0 < Q) {
            const uint64_t i0 = host_bitrev(g, logGq);
            // 1/((x-1)(x-w_h^-1)) depends on the domain only: cached per shape in the context
            char key[64];
            std::snprintf(key, sizeof key, "qsel_%u_%u_%llu_%u", log_h, logQ, (unsigned long long)i0, logGq);
            Fr* inv_den;
            auto it = ctx->ptabs.find(key);
            if (it != ctx->ptabs.end()) {
                inv_den = const_cast<Fr*>(it->second);
            } else {
                Fr* den = ctx->fbuf("q_den", Sq);
                inv_den = ctx->fbuf(key, Sq);
                LSP_HIP(launch_selector_denoms(tabQ, L1Q, GEN, wh_inv, Sq, den, st, i0, logGq));
                LSP_HIP(launch_batch_inverse(den, inv_den, Sq, st, ctx->bi_scratch(Sq)));
                ctx->ptabs[key] = inv_den;
            }
            {
                const Fr gh = fr_pow_u64(GEN, h), gq = host_two_adic_generator(log_q);
                Fr x = one;
                for (size_t k = 0; k < q; ++k) {
                    zh[k] = fr_sub(fr_mul(gh, x), one);
                    izh[k] = host_inv_cached(zh[k]);
                    x = fr_mul(x, gq);
                }
            }
            Fr* dzh = ctx->fbuf("q_zh", 2 * q);
            zh.insert(zh.end(), izh.begin(), izh.end());
            ctx->h2d_async("q_zh_h", dzh, zh.data(), 2 * q * sizeof(Fr));
            int32_t* dair = (int32_t*)ctx->buf("air", air.raw.size() * sizeof(int32_t));
            ctx->h2d_async("air_h", dair, air.raw.data(), air.raw.size() * sizeof(int32_t));
            qa.lde = lde;
            qa.w = (uint32_t)w;
            qa.logQ = logQ;
            qa.log_q = log_q;
            qa.air = dair;
            qa.air_len = (uint32_t)air.raw.size();
            qa.pub_alpha = pub[0];
            qa.pub_delta = pub[1];
            qa.gen = GEN;
            qa.wh_inv = wh_inv;
            qa.tabQ = tabQ;
            qa.L1 = L1Q;
            qa.zh = dzh;
            qa.inv_zh = dzh + q;
            qa.inv_den = inv_den;
            qa.out = qloc;
            qa.i0 = i0;
            qa.log_step = logGq;
            qa.row0 = row0;
            qa.n = Sq;
            qa.lde_next = lde_next;
            qa.row0_next = row0_next;
            qa.lde_rows = S;
            qa.lde_next_rows = lde_next ? S : 0;
        }

        // Constraints before alpha (round 4): every constraint C_j at this rank's
        // points depends on the trace LDE and the public values only; alpha enters
        // as the fold sum_j alpha^(n-1-j) C_j (air/src/lib.rs:116-167 through the
        // folder).  So the constraint values are evaluated on a low-priority side
        // stream once the trace tree's wide levels are done, beside its narrow
        // levels and the host's tree top, where most SIMDs idle; after alpha one
        // short kernel folds them.  For shapes whose evaluation outgrows that window
        // (ncons x points > 2^23: 2^20 rows and up at q = 4, the wide AIRs) the
        // quotient stays one kernel after alpha.  LSP_QUOTIENT_EARLY=0 / 1: never /
        // always (read per proof).
        bool early = false;
        const uint32_t ncons = (uint32_t)air.stats(ctx->public_degree).second;
        if (row0 < Q && !sub && ncons > 0) {
            const char* e = std::getenv("LSP_QUOTIENT_EARLY");
            early = e && *e ? *e != '0' : (uint64_t)ncons * Sq <= (1ull << 23);
        }
        struct SideJoin {  // the main stream never runs ahead of side work it did not wait for
            lsp_ctx* ctx;
            bool on = false;
            ~SideJoin() {
                if (on) (void)hipStreamWaitEvent(ctx->stream, ctx->ev_side, 0);
            }
        } side_join{ctx};
        std::function<void(hipEvent_t)> side_fn;
        if (early) {
            hipStream_t s2 = ctx->side();
            qa.cons = (uint32_t*)ctx->buf("q_cons", (size_t)ncons * 9 * Sq * sizeof(uint32_t));
            qa.ncons = ncons;
            side_fn = [&, s2](hipEvent_t ev) {
                LSP_HIP(hipStreamWaitEvent(s2, ev, 0));
                LSP_HIP(launch_quotient(qa, s2));
                LSP_HIP(hipEventRecord(ctx->ev_side, s2));
                side_join.on = true;
            };
        }

        Fr* tlay = ctx->fbuf("t_tree", 2 * S - 1);
        std::vector<std::vector<Fr>> ttop, qtop;
        T.begin("merkle tree");
        proof->troot = shard_root(ctx, comm,
                                  commit_device(ctx, one_mat(lde, (uint32_t)w), S, tlay, nullptr, early ? &side_fn : nullptr),
                                  ttop, "trace subtree roots");
        T.end("merkle tree");
        T.end("commit to trace data");

        // U7: the instance, then the quotient challenge (TranscriptCfg switches)
        const TranscriptCfg& TC = ctx->transcript;
        Challenger ch(&ctx->p2, TC.mont_bits);
        if (TC.log_degree) ch.observe(fr_from_u64(log_h));
        ch.observe(proof->troot);
        if (TC.public_values)
            for (size_t i = 0; i < npub; ++i) ch.observe(pub[i]);
        const Fr alpha = ch.sample();

        // ---- quotient: the constraint fold by alpha, divided by Z_H
        T.begin("compute quotient polynomial");
        if (row0 < Q) {
            qa.alpha = alpha;
            if (early) {
                LSP_REQUIRE(side_join.on, LSP_E_STATE, "the constraint evaluation was not issued");
                LSP_HIP(hipStreamWaitEvent(st, ctx->ev_side, 0));
                side_join.on = false;
                LSP_HIP(launch_quotient_fold(qa, st));
            } else {
                LSP_HIP(launch_quotient(qa, st));
            }
        }
        if (G > 1) {
            // rank r < Gq holds chunks j = bitrev(r) + Gq c as an h x cpr matrix: one
            // broadcast per holder (only the Gq holders send: Gq/G of an allgather's bytes).
            // split: the holder sends its chunks' coefficients (its own inverse
            // NTT), and no rank inverts the whole h x q matrix
            if (qsplit && g < Gq)
                LSP_HIP(launch_intt(qloc, ColMap::plain((uint32_t)cpr), stage + (size_t)g * Sq, cpr, log_h,
                                    ctx->twiddle29(log_h, true), st));
            for (uint32_t r = 0; r < Gq; ++r)
                comm.bcast(ctx, stage + (size_t)r * Sq, Sq * sizeof(Fr), (int)r,
                           qsplit ? "quotient chunk coefficients" : "quotient values");
            if (!qsplit) LSP_HIP(launch_assemble_chunks(stage, logGq, Sq, qv, st));
        }
        T.end("compute quotient polynomial");

        // ---- commit to quotient chunks: qv is the h x q matrix of chunks
        T.begin("commit to quotient poly chunks");
        const Fr gQ = host_two_adic_generator(logQ), gQinv = host_inv_cached(gQ);
        {
            Fr s = one;
            for (size_t j = 0; j < q; ++j) {
                shifts[j] = s;  // GEN / (GEN * w_Q^j)
                s = fr_mul(s, gQinv);
            }
        }
        Fr* qlde = ctx->fbuf("q_lde", S * q);
        T.begin("coset_lde_batch (quotient)");
        for (size_t j = 0; j < q; ++j) span("coset_lde_batch", 1, h, (int)lb);  // one launch, q independent columns
        if (qsplit) {  // the chunk coefficients straight from the exchange buffer (column j in slot bitrev(j mod Gq))
            lde_coeffs_device(ctx, stage, ColMap::blocked(logGq, (uint32_t)cpr), h, q, lb, shifts.data(), qlde, k0, nk);
        } else if (sub) {
            Fr* qc = ctx->fbuf("q_coef", h * q);
            LSP_HIP(launch_intt(qv, ColMap::plain((uint32_t)q), qc, q, log_h, ctx->twiddle29(log_h, true), st));
            subcoset_lde(ctx, qc, ColMap::plain((uint32_t)q), h, q, logN, b, g, shifts.data(), qlde, "q_sub");
        } else {
            lde_device(ctx, qv, h, q, lb, shifts.data(), qlde, k0, nk);
        }
        T.end("coset_lde_batch (quotient)");
        Fr* qlay = ctx->fbuf("q_tree", 2 * S - 1);
        proof->qroot = shard_root(ctx, comm, commit_device(ctx, one_mat(qlde, (uint32_t)q), S, qlay), qtop,
                                  "quotient subtree roots");
        T.end("commit to quotient poly chunks");
        ch.observe(proof->qroot);
        const Fr zeta = ch.sample();
        const Fr zeta_next = fr_mul(zeta, wh);

        // ---- open (alpha_fri is sampled once the opened values exist: U7 may
        // observe them first; the default samples it right after zeta, and
        // nothing touches the transcript in between)
        T.begin("open");
        T.begin("compute_inverse_denominators");
        uint32_t L1N;
        const Fr* tabN = pow_table(ctx, "tabN", host_two_adic_generator(logN), logN, L1N);
        Fr* dtmp = ctx->fbuf("o_den", S);
        Fr* inv_z = ctx->fbuf("o_invz", S);
        Fr* inv_zn = ctx->fbuf("o_invzn", S);
        LSP_HIP(launch_open_denoms(zeta, GEN, tabN, L1N, logN, S, dtmp, st, row0));
        // this rank's rows are the coset c H_S (c = GEN w_N^bitrev(row0)), so the
        // product of its denominators is prod (zeta - c w) = zeta^S - c^S: its
        // inverse on the host replaces the batch inverse's Fermat chain on the GPU
        const Fr cS = fr_pow_u64(fr_mul(GEN, fr_pow_u64(host_two_adic_generator(logN), host_bitrev(row0, logN))), S);
        const Fr den_prod = fr_sub(fr_pow_u64(zeta, S), cS);
        LSP_REQUIRE(!fr_is_zero(den_prod), LSP_E_STATE, "zeta lies in the LDE domain");
        const Fr den_prod_inv = fr_inv(den_prod);
        LSP_HIP(launch_batch_inverse(dtmp, inv_z, S, st, ctx->bi_scratch(S), &den_prod_inv));
        if (sub) {
            // x w_h^-1 leaves a sub-coset (w_h is not in H_S): the zeta_next
            // denominators are inverted on their own
            const Fr dpn = fr_sub(fr_pow_u64(zeta_next, S), cS);
            LSP_REQUIRE(!fr_is_zero(dpn), LSP_E_STATE, "zeta * w_h lies in the LDE domain");
            const Fr dpn_inv = fr_inv(dpn);
            LSP_HIP(launch_open_denoms(zeta_next, GEN, tabN, L1N, logN, S, dtmp, st, row0));
            LSP_HIP(launch_batch_inverse(dtmp, inv_zn, S, st, ctx->bi_scratch(S), &dpn_inv));
        } else {
            LSP_HIP(launch_shift_inverse(inv_z, inv_zn, wh_inv, logN, 1ull << lb, row0, S, st));
        }
        T.end("compute_inverse_denominators");
        T.begin("compute opened values with Lagrange interpolation");
        // Barycentric sums over one coset c H_h of the LDE domain: p(z) =
        // (z^h - c^h) / (h c^h) * sum_i p(x_i) x_i / (z - x_i).  Any coset gives
        // the same (unique) value, so with whole cosets per rank the three jobs
        // (trace at zeta, trace at zeta*w_h, the chunks at zeta) go to the ranks
        // that evaluated no quotient points (g >= Gq), each over its first coset,
        // instead of all to rank 0; an allgather of the values replaces rank 0's
        // broadcast.  sub: the low coset's h / S ranks add partial sums.
        const size_t maxw = std::max(w, q);
        const size_t nsum = 2 * w + q;
        Fr* sums = ctx->fbuf("o_sums", nsum);
        const size_t nlow = std::min(S, h);  // this rank's rows of one coset
        const size_t joff[3] = {0, w, 2 * w}, jw[3] = {w, w, q};
        bool job_here[3] = {false, false, false};
        if (sub) {
            job_here[0] = job_here[1] = job_here[2] = row0 < h;  // ranks 0 .. h/S - 1: the low coset's partial sums
        } else {
            const uint32_t nfree = G > Gq ? (uint32_t)(G - Gq) : 0u;
            for (int j = 0; j < 3; ++j)
                job_here[j] = g == (nfree ? G - 1 - (uint32_t)j % nfree : G - 1 - (uint32_t)j % G);
        }
        if (job_here[0] || job_here[1] || job_here[2]) {
            Fr* partial = ctx->fbuf("o_partial", ((nlow + 1023) / 1024) * maxw);
            const Fr* jm[3] = {lde, lde, qlde};
            const Fr* jinv[3] = {inv_z, inv_zn, inv_z};
            for (int j = 0; j < 3; ++j) {
                if (!job_here[j]) continue;
                uint32_t nb = 0;
                LSP_HIP(launch_interp_partial(jm[j], (uint32_t)jw[j], nlow, jinv[j], GEN, tabN, L1N, logN, partial, &nb,
                                              st, row0));
                LSP_HIP(launch_sum_partials(partial, nb, (uint32_t)jw[j], sums + joff[j], st));
            }
        }
        Fr* hs = (Fr*)ctx->hbuf("o_sums_h", nsum * sizeof(Fr));  // pinned
        if (job_here[0] || job_here[1] || job_here[2]) {
            LSP_HIP(hipMemcpyAsync(hs, sums, nsum * sizeof(Fr), hipMemcpyDeviceToHost, st));
            LSP_HIP(hipStreamSynchronize(st));
        }
        // the coset of this rank's first rows: c = GEN w_N^bitrev(row0) (sub: the low coset, GEN)
        const Fr cpos = sub ? GEN : fr_mul(GEN, fr_pow_u64(host_two_adic_generator(logN), host_bitrev(row0, logN)));
        const Fr ch_ = fr_pow_u64(cpos, h);
        const Fr dinv = host_inv_cached(fr_mul(ch_, fr_from_u64(h)));
        auto factor = [&](const Fr& z) { return fr_mul(fr_sub(fr_pow_u64(z, h), ch_), dinv); };
        const Fr jz[3] = {zeta, zeta_next, zeta};
        for (int j = 0; j < 3; ++j) {
            const Fr f = factor(jz[j]);
            for (size_t k = 0; k < jw[j]; ++k) hs[joff[j] + k] = job_here[j] ? fr_mul(hs[joff[j] + k], f) : fr_zero();
        }
        if (G > 1) {  // every value from its job's rank(s): the sum over ranks
            const std::vector<Fr> all = comm.allgather_fr(ctx, hs, nsum, "opened values");
            for (size_t k = 0; k < nsum; ++k) {
                Fr acc = fr_zero();
                for (uint32_t r = 0; r < G; ++r) acc = fr_add(acc, all[(size_t)r * nsum + k]);
                hs[k] = acc;
            }
        }
        proof->tl.assign(hs, hs + w);
        proof->tn.assign(hs + w, hs + 2 * w);
        proof->qc.assign(hs + 2 * w, hs + 2 * w + q);
        T.end("compute opened values with Lagrange interpolation");
        if (TC.opened_values) {  // U7: every opened value, in (matrix, point) order, before alpha_fri
            for (const Fr& v : proof->tl) ch.observe(v);
            for (const Fr& v : proof->tn) ch.observe(v);
            for (const Fr& v : proof->qc) ch.observe(v);
        }
        const Fr alpha_fri = ch.sample();

        T.begin("reduce rows");
        // the (matrix, point) order of TwoAdicFriPcs::open that the reduction
        // below folds in (k_reduce_rows): trace at zeta, trace at zeta*w_h,
        // then quotient chunk j at zeta
        span("reduce matrix quotient", w, N, -1);
        span("reduce matrix quotient", w, N, -1);
        for (size_t j = 0; j < q; ++j) span("reduce matrix quotient", 1, N, -1);
        std::vector<Fr> apw(2 * w + q);
        apw[0] = one;
        for (size_t k = 1; k < apw.size(); ++k) apw[k] = fr_mul(apw[k - 1], alpha_fri);
        Fr ry_z = fr_zero(), ry_zn = fr_zero();
        for (size_t c = 0; c < w; ++c) {
            ry_z = fr_add(ry_z, fr_mul(apw[c], proof->tl[c]));
            ry_zn = fr_add(ry_zn, fr_mul(apw[c], proof->tn[c]));
        }
        Fr* dapw = ctx->fbuf("o_apw", apw.size() + q);
        const size_t napw = apw.size();
        apw.insert(apw.end(), proof->qc.begin(), proof->qc.end());
        ctx->h2d_async("o_apw_h", dapw, apw.data(), apw.size() * sizeof(Fr));
        // FRI vectors: this rank's slice of round r's input (length (N >> r) / G), back to back
        Fr* fvec = ctx->fbuf("f_vec", 2 * S);
        ReduceArgs ra;
        ra.lde = lde;
        ra.w = (uint32_t)w;
        ra.qlde = qlde;
        ra.q = (uint32_t)q;
        ra.inv_z = inv_z;
        ra.inv_zn = inv_zn;
        ra.apw = dapw;
        ra.ry_z = ry_z;
        ra.ry_zn = ry_zn;
        ra.ryq = dapw + napw;
        ra.out = fvec;
        ra.n = S;
        ra.lds_max = ctx->lds_per_block;
        if (const size_t nsc = reduce_rows_scratch(ra.w, ra.q, ra.lds_max))  // constants beyond the LDS: global
            ra.consts29 = (F29*)ctx->buf("o_rr_consts", nsc * sizeof(F29));
        LSP_HIP(launch_reduce_rows(ra, st));
        T.end("reduce rows");

        // ---- FRI commit phase
        T.begin("FRI prover");
        T.begin("commit phase");
        const size_t final_len = (size_t)1 << (lb + ctx->log_final_poly_len);
        struct FriRound {
            const Fr* vec;   // this rank's copy of the round's input (its slice when sharded)
            const Fr* tree;  // layers of this rank's (sub)tree
            size_t ml;       // leaves of that (sub)tree
            bool sharded;
            std::vector<std::vector<Fr>> top;
        };
        std::vector<FriRound> rounds;
        // shortest slice worth a collective per round (tests lower it to shard every round)
        size_t FRI_SHARD_MIN = (size_t)1 << 12;
        if (const char* e = std::getenv("LSP_FRI_SHARD_MIN")) FRI_SHARD_MIN = std::max<size_t>(1, std::strtoull(e, nullptr, 10));
        Fr* ftree = ctx->fbuf("f_tree", 2 * S + 2 * (size_t)G * FRI_SHARD_MIN);
        Fr* fv = fvec;
        size_t len = N, vo = 0, to = 0;
        bool sharded = G > 1;
        const Fr half = host_inv_cached(fr_from_u64(2));
        auto replicate = [&]() {  // gather the short vector to every rank
            const size_t loc = len >> b;
            Fr* rep = ctx->fbuf("f_rep", 2 * len);
            comm.allgather(ctx, fv + vo, rep, loc * sizeof(Fr), "FRI vector");
            fv = rep;
            vo = 0;
            sharded = false;
        };
        // round r's fold (by beta_r) runs fused into round r+1's leaf hashing
        FoldSpec pend{};
        size_t pend_m = 0;  // folded values (this rank's slice)
        bool pending = false;
        auto flush_fold = [&]() {
            if (!pending) return;
            LSP_HIP(launch_fri_fold(pend.v, pend_m, pend.half, pend.half_beta, pend.tab, pend.L1,
                                    pend.vout, st, pend.i0, (int)pend.logm));
            pending = false;
        };
        size_t host_tail = ctx->fri_host_tail;
        if (const char* e = std::getenv("LSP_FRI_HOST_TAIL")) host_tail = std::strtoull(e, nullptr, 10);
        const Fr* hfin = nullptr;  // the final vector, when the host ran the last rounds
        while (len > final_len) {
            if (sharded && (len >> b) < 2 * FRI_SHARD_MIN) {
                flush_fold();  // the gathered vector must exist
                replicate();
            }
            if (!sharded && len / 2 <= host_tail) {
                // The last rounds wholly on the host: their trees are a few thousand
                // permutations in a chain of short levels (~58 us each on the GPU, a few
                // us on the host pool).  One download of the vector; per round the host
                // hashes the tree, samples beta and folds; the layers and folded vectors
                // go back asynchronously for the query openings, which gather on the device.
                flush_fold();
                const auto th0 = std::chrono::steady_clock::now();
                size_t hn = final_len, ht = 0;
                for (size_t l = len; l > final_len; l /= 2) {
                    hn += l;
                    ht += l - 1;
                }
                Fr* hv = (Fr*)ctx->hbuf("fri_tail", (hn + ht) * sizeof(Fr));
                Fr* htr = hv + hn;
                LSP_HIP(hipMemcpyAsync(hv, fv + vo, len * sizeof(Fr), hipMemcpyDeviceToHost, st));
                LSP_HIP(hipStreamSynchronize(st));
                const auto th1 = std::chrono::steady_clock::now();
                const size_t rounds_gpu = rounds.size();
                HostPool& pool = ctx->host_pool();
                size_t hvo = 0, hto = 0;
                const size_t to0 = to, vo0 = vo, len0 = len;
                while (len > final_len) {
                    const size_t m = len / 2;
                    const uint32_t logm = log2_exact(m);
                    const Fr* v = hv + hvo;
                    Fr* lay = htr + hto;
                    const auto tr0 = std::chrono::steady_clock::now();
                    // leaves (a 2-element leaf's hash_iter is compress, A4/A5) and levels in one pass
                    auto tr1 = tr0;
                    const size_t end = host_levels(ctx, lay, m, &tr1, v);
                    const auto tr2 = std::chrono::steady_clock::now();
                    FriRound R;
                    R.vec = fv + vo;
                    R.tree = ftree + to;
                    R.ml = m;
                    R.sharded = false;
                    const Fr root = lay[end - 1];
                    proof->roots.push_back(root);
                    ch.observe(root);
                    const Fr hb = fr_mul(ch.sample(), half);
                    std::vector<Fr>& tw = ctx->fold_tw[logm];  // g^-bitrev(i), g = w_{2m}
                    if (tw.size() != m) {
                        const Fr ginv = host_inv_cached(host_two_adic_generator(logm + 1));
                        std::vector<Fr> pw(m);
                        pw[0] = one;
                        for (size_t j = 1; j < m; ++j) pw[j] = fr_mul(pw[j - 1], ginv);
                        tw.resize(m);
                        for (size_t i = 0; i < m; ++i) tw[i] = pw[host_bitrev(i, logm)];
                    }
                    Fr* out = hv + hvo + len;
                    // half (v0 + v1) + hb g^-bitrev(i) (v0 - v1), in the 64-bit lazy
                    // form; short vectors on this thread (a pool round trip costs more)
                    const hp64::F hh = hp64::from(half), hbb = hp64::from(hb);
                    auto fold_blk = [&](size_t i0, size_t i1) {
                        for (size_t i = i0; i < i1; ++i) {
                            const hp64::F a = hp64::from(v[2 * i]), b = hp64::from(v[2 * i + 1]);
                            const hp64::F p = hp64::mul(hbb, hp64::from(tw[i]));
                            out[i] = hp64::to_canonical(hp64::add(hp64::mul(hh, hp64::add(a, b)),
                                                                  hp64::mul(p, hp64::sub(a, b))));
                        }
                    };
                    if (m <= 256)
                        fold_blk(0, m);
                    else
                        pool.parallel_for((m + 63) / 64, [&](size_t blk) { fold_blk(64 * blk, std::min(m, 64 * blk + 64)); });
                    if (g_top_times.on) {
                        const auto tr3 = std::chrono::steady_clock::now();
                        auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
                            return std::chrono::duration<double, std::micro>(b - a).count();
                        };
                        std::fprintf(stderr, "[fri tail round] m %5zu  leaves %6.1f  levels %6.1f  challenge+fold+copies %6.1f us\n",
                                     m, us(tr0, tr1), us(tr1, tr2), us(tr2, tr3));
                    }
                    rounds.push_back(std::move(R));
                    hvo += len;
                    vo += len;
                    hto += end;
                    to += end;
                    len = m;
                }
                hfin = hv + hvo;
                // every round's layers and folded vector back to the device (for the
                // query gather): both are contiguous, so two copies instead of two per round
                LSP_HIP(hipMemcpyAsync(ftree + to0, htr, (to - to0) * sizeof(Fr), hipMemcpyHostToDevice, st));
                LSP_HIP(hipMemcpyAsync(fv + vo0 + len0, hv + len0, (hvo + len - len0) * sizeof(Fr), hipMemcpyHostToDevice, st));
                if (g_top_times.on)
                    std::fprintf(stderr, "[fri tail] %zu rounds on the host: %.1f us (download %.1f us)\n",
                                 rounds.size() - rounds_gpu,
                                 std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - th0).count(),
                                 std::chrono::duration<double, std::micro>(th1 - th0).count());
                break;
            }
            const size_t m = len / 2, ml = sharded ? (m >> b) : m;
            FriRound R;
            R.vec = fv + vo;
            R.tree = ftree + to;
            R.ml = ml;
            R.sharded = sharded;
            const Fr lroot = commit_device(ctx, one_mat(fv + vo, 2), ml, ftree + to, pending ? &pend : nullptr);
            pending = false;
            const Fr root = sharded ? shard_root(ctx, comm, lroot, R.top, "FRI subtree roots") : lroot;
            proof->roots.push_back(root);
            ch.observe(root);
            const Fr beta = ch.sample();
            uint32_t L1F;
            const uint32_t logm = log2_exact(m);
            const Fr ginv = host_inv_cached(host_two_adic_generator(logm + 1));
            const Fr* tabF = pow_table(ctx, "tabF", ginv, logm, L1F);
            pend.v = fv + vo;
            pend.vout = fv + vo + 2 * ml;
            pend.half = half;
            pend.half_beta = fr_mul(beta, half);
            pend.tab = tabF;
            pend.L1 = L1F;
            pend.logm = logm;
            pend.i0 = sharded ? (uint64_t)g * ml : 0;
            pend_m = ml;
            pending = true;
            rounds.push_back(std::move(R));
            vo += 2 * ml;
            to += 2 * ml - 1;
            len = m;
        }
        flush_fold();
        if (sharded) replicate();
        std::vector<Fr> fin(len);
        if (hfin)
            std::copy(hfin, hfin + len, fin.begin());
        else {
            Fr* hf = (Fr*)ctx->hbuf("f_final_h", len * sizeof(Fr));
            LSP_HIP(hipMemcpyAsync(hf, fv + vo, len * sizeof(Fr), hipMemcpyDeviceToHost, st));
            LSP_HIP(hipStreamSynchronize(st));
            std::copy(hf, hf + len, fin.begin());
        }
        T.end("commit phase");
        {
            // final poly: bit-reverse, IDFT (naive, len <= 2^lb small), truncate
            span("divide_by_height", 1, len, -1);
            const uint32_t lgl = log2_exact(len);
            std::vector<Fr> br(len);
            for (size_t i = 0; i < len; ++i) br[i] = fin[host_bitrev(i, lgl)];
            const Fr winv = host_inv_cached(host_two_adic_generator(lgl));
            const Fr linv = host_inv_cached(fr_from_u64(len));
            const size_t flen = (size_t)1 << ctx->log_final_poly_len;
            for (size_t k = 0; k < len; ++k) {
                Fr acc = fr_zero();
                const Fr wk = fr_pow_u64(winv, k);
                Fr p = one;
                for (size_t j = 0; j < len; ++j) {
                    acc = fr_add(acc, fr_mul(br[j], p));
                    p = fr_mul(p, wk);
                }
                acc = fr_mul(acc, linv);
                if (k < flen)
                    proof->final_poly.push_back(acc);
                else  // (a rehearsal rank's fabricated peer data folds to no polynomial: not checked)
                    LSP_REQUIRE(fr_is_zero(acc) || comm.rehearsal(), LSP_E_STATE, "FRI final polynomial degree too high");
            }
            if (TC.final_poly)  // U12
                for (const Fr& c : proof->final_poly) ch.observe(c);
        }
        T.begin("grind for proof-of-work witness");
        proof->pow_w = fr_from_u64(grind_device(ctx, ch, ctx->pow_bits));
        T.end("grind for proof-of-work witness");

        // ---- query phase: the owner of a query's row (rank idx / S) gathers the
        // openings below the rank subtrees in one kernel; the layers above come
        // from the host top trees every rank holds.
        flush_top_uploads(ctx);  // the gather below reads the tree tops
        T.begin("query phase");
        const auto q0 = std::chrono::steady_clock::now();
        const uint32_t nr = (uint32_t)rounds.size();
        const uint32_t nq = ctx->num_queries;
        std::vector<size_t> idxs(nq);
        for (uint32_t qi = 0; qi < nq; ++qi) idxs[qi] = (size_t)ch.sample_bits(logN);
        const auto q1 = std::chrono::steady_clock::now();
        size_t E = w + logS + q + logS;  // elements per query below the rank subtrees
        for (const FriRound& R : rounds) E += 1 + log2_exact(R.ml);
        std::vector<uint64_t> ptrs;
        std::vector<uint32_t> mine;
        for (uint32_t qi = 0; qi < nq; ++qi) {
            const size_t idx = idxs[qi];
            if ((idx >> logS) != g) continue;
            mine.push_back(qi);
            const size_t li = idx - row0;
            auto P = [&](const Fr* p) { ptrs.push_back((uint64_t)(uintptr_t)p); };
            auto path = [&](const Fr* lay, size_t leaves, size_t leaf) {
                size_t off = 0, ln = leaves;
                for (uint32_t i = 0; (1ull << i) < leaves; ++i) {
                    P(lay + off + ((leaf >> i) ^ 1));
                    off += ln;
                    ln >>= 1;
                }
            };
            for (size_t c = 0; c < w; ++c) P(lde + li * w + c);
            path(tlay, S, li);
            for (size_t j = 0; j < q; ++j) P(qlde + li * q + j);
            path(qlay, S, li);
            for (uint32_t r = 0; r < nr; ++r) {
                const FriRound& R = rounds[r];
                const size_t ii = idx >> r;                           // global index in round r's vector
                const size_t base = R.sharded ? (size_t)g * 2 * R.ml : 0;  // global index of R.vec[0]
                P(R.vec + ((ii ^ 1) - base));
                path(R.tree, R.ml, (ii >> 1) - base / 2);
            }
        }
        LSP_REQUIRE(ptrs.size() == mine.size() * E, LSP_E_STATE, "query opening layout mismatch");
        // one rank: every query is this rank's, in order, so the gathered openings
        // are already the all-ranks layout and the records read them in place
        // (two host copies of ~E * nq elements fewer between proofs)
        const bool in_place = G == 1;
        std::vector<Fr> slots(in_place ? 0 : (size_t)nq * E, fr_zero());
        const Fr* opened = nullptr;  // the openings of every query, (owner rank, query)-major
        if (!ptrs.empty()) {
            // the gather reads its pointer list from pinned host memory and writes the
            // openings into coherent pinned memory: no copy either side of the kernel
            // (LSP_GATHER_ZEROCOPY=0: upload, gather to HBM, download; read per call)
            const char* zc = std::getenv("LSP_GATHER_ZEROCOPY");
            Fr* got;
            if (!(zc && *zc == '0')) {
                uint64_t* hp = (uint64_t*)ctx->hbuf("g_ptrs_zc", ptrs.size() * sizeof(uint64_t));
                std::memcpy(hp, ptrs.data(), ptrs.size() * sizeof(uint64_t));
                got = (Fr*)ctx->hbuf("g_out_zc", ptrs.size() * sizeof(Fr), hipHostMallocCoherent);
                LSP_HIP(launch_gather(hp, got, ptrs.size(), st));
            } else {
                uint64_t* dptrs = (uint64_t*)ctx->buf("g_ptrs", ptrs.size() * sizeof(uint64_t));
                Fr* dgot = ctx->fbuf("g_out", ptrs.size());
                ctx->h2d_async("g_ptrs_h", dptrs, ptrs.data(), ptrs.size() * sizeof(uint64_t));
                LSP_HIP(launch_gather(dptrs, dgot, ptrs.size(), st));
                got = (Fr*)ctx->hbuf("g_out_h", ptrs.size() * sizeof(Fr));  // pinned: no staging copy
                LSP_HIP(hipMemcpyAsync(got, dgot, ptrs.size() * sizeof(Fr), hipMemcpyDeviceToHost, st));
            }
            LSP_HIP(hipStreamSynchronize(st));
            if (in_place)
                opened = got;
            else
                for (size_t k = 0; k < mine.size(); ++k)
                    std::copy(got + k * E, got + (k + 1) * E, slots.begin() + (size_t)mine[k] * E);
        }
        const auto q2 = std::chrono::steady_clock::now();
        std::vector<Fr> all;
        if (!in_place) {
            all = comm.allgather_fr(ctx, slots.data(), slots.size(), "query openings");
            opened = all.data();
        }
        LSP_REQUIRE(opened || nq == 0, LSP_E_STATE, "query openings missing");
        auto top_path = [&](const std::vector<std::vector<Fr>>& top, size_t sub, std::vector<Fr>& out) {
            for (uint32_t i = 0; i + 1 < top.size(); ++i) out.push_back(top[i][(sub >> i) ^ 1]);
        };
        // each query's record is independent: assembled (and below serialized)
        // on the host pool -- ~0.1 + 0.2 ms of one thread's time at 2^19
        // records of a freed proof keep their vectors' capacity (proof_release)
        proof->queries = recycled_queries();
        proof->queries.resize(nq);
        const char* qp = std::getenv("LSP_QUERY_POOL");  // =0: one thread, wire bytes on demand (A/B)
        const bool qpool = !(qp && *qp == '0');
        HostPool serial_pool(0);
        (qpool ? ctx->host_pool() : serial_pool).parallel_for(nq, [&](size_t qi) {
            const size_t idx = idxs[qi], o = idx >> logS;
            const Fr* e = opened + (o * nq + qi) * E;
            lsp_query& qq = proof->queries[qi];
            qq.sib.clear();
            qq.sib.reserve(nr);
            qq.fpath.resize(nr);
            qq.trow.assign(e, e + w);
            e += w;
            qq.tpath.assign(e, e + logS);
            e += logS;
            top_path(ttop, o, qq.tpath);
            qq.qrow.assign(e, e + q);
            e += q;
            qq.qpath.assign(e, e + logS);
            e += logS;
            top_path(qtop, o, qq.qpath);
            for (uint32_t r = 0; r < nr; ++r) {
                const FriRound& R = rounds[r];
                qq.sib.push_back(*e++);
                const uint32_t lg = log2_exact(R.ml);
                std::vector<Fr>& pth = qq.fpath[r];
                pth.assign(e, e + lg);
                e += lg;
                if (R.sharded) top_path(R.top, o, pth);
            }
        });
        // the wire bytes now, in parallel (lsp_proof_serialize returns the cached copy)
        if (qpool) {
            std::vector<uint8_t> buf = recycled_wire();
            proof->wire = serialize(*proof, &ctx->host_pool(), &buf);
        }
        const auto q3 = std::chrono::steady_clock::now();
        T.end("query phase");
        T.end("FRI prover");
        T.end("open");
        T.end("prove");
        T.collect();
        if (g_top_times.on) {
            const auto q4 = std::chrono::steady_clock::now();
            auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
            std::fprintf(stderr, "[query] samples %.1f us, gather+sync %.1f us, assemble %.1f us, collect %.1f us; "
                                 "entry -> LDE issued %.1f us\n",
                         us(q0, q1), us(q1, q2), us(q2, q3), us(q3, q4), us(t_entry, t_lde_issued));
        }
    } catch (...) {
        delete proof;
        throw;
    }
    return proof;
}

lsp_proof* prove_device(lsp_ctx* ctx, const Fr* d_trace, size_t h, size_t w, const Air& air, const Fr* pub,
                        size_t npub) {
    SoloComm solo;
    return prove_shard(ctx, solo, d_trace, h, w, air, pub, npub);
}

}  // namespace lsp
