// Host helpers: field constants, AIR descriptor parsing and symbolic degrees,
// device buffer pool, twiddle cache.
#include "host.hpp"

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdlib>
#include <cstring>

#if defined(__linux__)
#include <sched.h>
#endif

namespace lsp {

Fr host_generator() { return fr_from_u64(22); }

Fr host_inv_cached(const Fr& a) {
    static std::mutex mu;
    static std::map<std::array<uint32_t, 8>, Fr> cache;
    std::array<uint32_t, 8> k;
    for (int i = 0; i < 8; ++i) k[i] = a.v[i];
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find(k);
        if (it != cache.end()) return it->second;
    }
    const Fr r = fr_inv(a);
    std::lock_guard<std::mutex> g(mu);
    if (cache.size() > 4096) cache.clear();
    cache[k] = r;
    return r;
}

Fr host_two_adic_generator(uint32_t bits) {
    // ROOT_2_47 = 22^((r-1) >> 47); (r-1) >> 47 as 32-bit words
    static Fr root47 = [] {
        // r - 1 = 0x12ab655e9a2ca55660b44d1e5c37b00159aa76fed00000010a11800000000000
        uint32_t e[8] = {0x00000000u, 0x0a118000u, 0xd0000001u, 0x59aa76feu,
                         0x5c37b001u, 0x60b44d1eu, 0x9a2ca556u, 0x12ab655eu};
        // shift right by 47 bits: one word (32) + 15 bits
        uint32_t s[8] = {0};
        for (int i = 0; i < 7; ++i) s[i] = e[i + 1];
        uint32_t t[8] = {0};
        for (int i = 0; i < 8; ++i) t[i] = (s[i] >> 15) | (i + 1 < 8 ? (s[i + 1] << 17) : 0u);
        Fr g = fr_from_u64(22), r = fr_one();
        bool started = false;
        for (int w = 7; w >= 0; --w)
            for (int k = 31; k >= 0; --k) {
                if (started) r = fr_sqr(r);
                if ((t[w] >> k) & 1u) {
                    r = started ? fr_mul(r, g) : g;
                    started = true;
                }
            }
        return r;
    }();
    if (bits > 47) throw LspError(LSP_E_SIZE, "two-adicity of Fr is 47");
    Fr r = root47;
    for (uint32_t k = bits; k < 47; ++k) r = fr_sqr(r);
    return r;
}

uint64_t host_bitrev(uint64_t x, uint32_t bits) {
    uint64_t r = 0;
    for (uint32_t i = 0; i < bits; ++i) {
        r = (r << 1) | (x & 1);
        x >>= 1;
    }
    return r;
}

uint32_t log2_exact(size_t n) {
    uint32_t b = 0;
    while (((size_t)1 << b) < n) ++b;
    if (n == 0 || ((size_t)1 << b) != n) throw LspError(LSP_E_SIZE, "height must be a power of two");
    return b;
}

HostPool::HostPool(unsigned workers) {
    for (unsigned i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
}

HostPool::~HostPool() {
    {
        std::lock_guard<std::mutex> lk(m_);
        stop_.store(true);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
}

static inline void cpu_relax() {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
}

void HostPool::loop() {
    uint64_t seen = 0;
    for (;;) {
        // spin for a new generation, then sleep
        const auto t0 = std::chrono::steady_clock::now();
        const int64_t until = std::max<int64_t>(
            std::chrono::duration_cast<std::chrono::nanoseconds>((t0 + std::chrono::microseconds(kSpinUs)).time_since_epoch())
                .count(),
            spin_until_ns_.load(std::memory_order_relaxed));
        for (unsigned it = 0; gen_.load() == seen && !stop_.load(); ++it) {
            cpu_relax();
            if ((it & 255) == 255 &&
                std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
                        .count() > until) {
                std::unique_lock<std::mutex> lk(m_);
                sleepers_.fetch_add(1);  // seq_cst: pairs with parallel_for's gen_ / sleepers_ order
                cv_.wait(lk, [&] { return stop_.load() || gen_.load() != seen; });
                sleepers_.fetch_sub(1);
                break;
            }
        }
        if (stop_.load()) return;
        seen = gen_.load();
        const auto* job = job_;
        const size_t n = n_;
        for (size_t i; (i = next_.fetch_add(1)) < n;) (*job)(i);
        busy_.fetch_sub(1);
    }
}

void HostPool::wake(unsigned spin_us) {
    if (th_.empty()) return;
    if (spin_us)
        spin_until_ns_.store(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                 (std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us)).time_since_epoch())
                                 .count(),
                             std::memory_order_relaxed);
    while (busy_.load() != 0) cpu_relax();
    job_ = nullptr;
    n_ = 0;
    next_.store(0);
    busy_.store((unsigned)th_.size());
    gen_.fetch_add(1);
    if (sleepers_.load() != 0) {
        std::lock_guard<std::mutex> lk(m_);
        cv_.notify_all();
    }
}

void HostPool::parallel_for(size_t n, const std::function<void(size_t)>& f) {
    if (th_.empty() || n < 2) {
        for (size_t i = 0; i < n; ++i) f(i);
        return;
    }
    while (busy_.load() != 0) cpu_relax();  // a wake() may still be draining
    // the previous job has fully drained (busy_ == 0), so no worker reads these
    job_ = &f;
    n_ = n;
    next_.store(0);
    busy_.store((unsigned)th_.size());
    gen_.fetch_add(1);
    if (sleepers_.load() != 0) {
        std::lock_guard<std::mutex> lk(m_);
        cv_.notify_all();
    }
    for (size_t i; (i = next_.fetch_add(1)) < n;) f(i);
    for (unsigned it = 0; busy_.load() != 0; ++it) {
        cpu_relax();
        if ((it & 4095) == 4095) std::this_thread::yield();
    }
}

Fr P2Host::hash(const Fr* in, size_t n) const {
    Fr s0 = fr_zero(), s1 = fr_zero(), s2 = fr_zero();
    size_t k = 0;
    while (k + 2 <= n) {
        s0 = in[k];
        s1 = in[k + 1];
        permute(s0, s1, s2);
        k += 2;
    }
    if (k < n) {
        s0 = in[k];
        permute(s0, s1, s2);
    }
    return s0;
}

// ------------------------------------------------------------------- AIR
Air Air::parse(const int32_t* d, size_t n) {
    Air air;
    LSP_REQUIRE(d && n >= 1, LSP_E_ARG, "empty AIR descriptor");
    air.raw.assign(d, d + n);
    size_t p = 0;
    auto next = [&]() -> int32_t {
        LSP_REQUIRE(p < n, LSP_E_ARG, "truncated AIR descriptor");
        return d[p++];
    };
    auto col = [&]() -> int32_t {
        int32_t c = next();
        LSP_REQUIRE(c >= 0 && c < (1 << 20), LSP_E_ARG, "bad column id in AIR descriptor");
        air.max_col = std::max(air.max_col, (uint32_t)c);
        return c;
    };
    const int32_t nc = next();
    LSP_REQUIRE(nc >= 1 && nc <= 4096, LSP_E_ARG, "bad config count in AIR descriptor");
    for (int32_t c = 0; c < nc; ++c) {
        AirCfg g;
        g.type = next();
        if (g.type == LSP_AIR_PERMUTATION) {
            const int32_t na = next(), nb = next();
            LSP_REQUIRE(na >= 1 && nb >= 1 && na <= 4096 && nb <= 4096, LSP_E_ARG, "bad permutation widths");
            for (int32_t i = 0; i < na; ++i) g.a.push_back(col());
            for (int32_t i = 0; i < nb; ++i) g.b.push_back(col());
            g.binv = col();
            g.check = col();
        } else if (g.type == LSP_AIR_LOOKUP) {
            const int32_t na = next();
            LSP_REQUIRE(na >= 1 && na <= 4096, LSP_E_ARG, "bad lookup A width");
            for (int32_t i = 0; i < na; ++i) g.a.push_back(col());
            g.ntab = next();
            g.nbc = next();
            LSP_REQUIRE(g.ntab >= 1 && g.nbc >= 1 && g.ntab <= 4096 && g.nbc <= 4096, LSP_E_ARG,
                        "bad lookup B tables");
            for (int32_t i = 0; i < g.ntab * g.nbc; ++i) g.b.push_back(col());
            g.a_filter = col();
            for (int32_t t = 0; t < g.ntab; ++t) g.b_filter.push_back(col());
            g.a_inv = col();
            for (int32_t t = 0; t < g.ntab; ++t) g.b_inv.push_back(col());
            for (int32_t t = 0; t < g.ntab; ++t) g.occ.push_back(col());
            g.check = col();
        } else {
            throw LspError(LSP_E_ARG, "unknown AIR config type");
        }
        air.cfgs.push_back(std::move(g));
    }
    LSP_REQUIRE(p == n, LSP_E_ARG, "trailing data in AIR descriptor");
    return air;
}

// Symbolic degree_multiple rules of p3-uni-stark: main variables 1,
// constants 0, public values `pd` (U6), IsFirstRow/IsLastRow 1,
// IsTransition 0; Add/Sub max, Mul sum.  Horner combos start from ZERO.
static int horner_deg(size_t n, int pd) {
    int d = 0;
    for (size_t i = 0; i < n; ++i) d = std::max(d + pd, 1);
    return d;
}

std::pair<int, int> Air::stats(int pd) const {
    int maxd = 0, k = 0;
    for (const auto& g : cfgs) {
        if (g.type == LSP_AIR_PERMUTATION) {
            const int a = std::max(horner_deg(g.a.size(), pd), pd), b = std::max(horner_deg(g.b.size(), pd), pd);
            maxd = std::max({maxd, b + 1, 1 + std::max(1, a + 1), std::max(1, a + 2), 2});
            k += 4;
        } else {
            const int a = std::max(horner_deg(g.a.size(), pd), pd);
            maxd = std::max(maxd, a + 1);
            const int bdeg = std::max(horner_deg((size_t)g.nbc, pd), pd);
            maxd = std::max(maxd, bdeg + 1);
            const int lc = 3;
            maxd = std::max({maxd, 1 + lc, lc, 2});
            k += 1 + g.ntab + 3;
        }
    }
    return {maxd, k};
}

uint32_t Air::log_quotient_degree(int pd) const {
    int d = std::max(stats(pd).first, 2);
    uint32_t lg = 0;
    while ((1 << lg) < d - 1) ++lg;
    return lg;
}

static Fr horner(const Fr* row, const int32_t* ids, size_t n, const Fr& a) {
    Fr acc = fr_zero();
    for (size_t i = 0; i < n; ++i) acc = fr_add(fr_mul(acc, a), row[ids[i]]);
    return acc;
}

void Air::eval_fold(const Fr* loc, const Fr* nxt, const Fr& ap, const Fr& dl, const Fr& first, const Fr& last,
                    const Fr& trans, const Fr& al, Fr& acc) const {
    const Fr one = fr_one();
    auto push = [&](const Fr& x) { acc = fr_add(fr_mul(acc, al), x); };
    for (const auto& g : cfgs) {
        if (g.type == LSP_AIR_PERMUTATION) {
            const Fr a_l = fr_add(horner(loc, g.a.data(), g.a.size(), ap), dl);
            const Fr b_l = fr_add(horner(loc, g.b.data(), g.b.size(), ap), dl);
            push(fr_sub(fr_mul(b_l, loc[g.binv]), one));
            push(fr_mul(first, fr_sub(loc[g.check], fr_mul(a_l, loc[g.binv]))));
            const Fr a_n = fr_add(horner(nxt, g.a.data(), g.a.size(), ap), dl);
            push(fr_mul(trans, fr_sub(nxt[g.check], fr_mul(fr_mul(loc[g.check], a_n), nxt[g.binv]))));
            push(fr_mul(last, fr_sub(loc[g.check], one)));
        } else {
            const Fr a_l = fr_add(horner(loc, g.a.data(), g.a.size(), ap), dl);
            push(fr_sub(fr_mul(a_l, loc[g.a_inv]), one));
            Fr lc = fr_mul(loc[g.a_filter], loc[g.a_inv]);
            Fr nc = fr_mul(nxt[g.a_filter], nxt[g.a_inv]);
            for (int32_t t = 0; t < g.ntab; ++t) {
                const Fr b_l = fr_add(horner(loc, g.b.data() + t * g.nbc, g.nbc, ap), dl);
                push(fr_sub(fr_mul(b_l, loc[g.b_inv[t]]), one));
                lc = fr_sub(lc, fr_mul(fr_mul(loc[g.b_filter[t]], loc[g.occ[t]]), loc[g.b_inv[t]]));
                nc = fr_sub(nc, fr_mul(fr_mul(nxt[g.b_filter[t]], nxt[g.occ[t]]), nxt[g.b_inv[t]]));
            }
            push(fr_mul(first, fr_sub(loc[g.check], lc)));
            push(fr_mul(trans, fr_sub(fr_sub(nxt[g.check], loc[g.check]), nc)));
            push(fr_mul(last, loc[g.check]));
        }
    }
}

}  // namespace lsp

// ------------------------------------------------------------------ context
void* lsp_ctx::buf(const std::string& name, size_t bytes) {
    Buf& b = pool[name];
    if (b.cap < bytes) {
        if (b.p) {
            LSP_HIP(hipStreamSynchronize(stream));
            LSP_HIP(hipFree(b.p));
            b.p = nullptr;
            b.cap = 0;
        }
        if (bytes) {
            hipError_t e = hipMalloc(&b.p, bytes);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                throw lsp::LspError(LSP_E_OOM, "hipMalloc(" + std::to_string(bytes) + ") for " + name + " failed");
            }
            b.cap = bytes;
        }
    }
    return b.p;
}

void lsp_ctx::release(const std::string& prefix) {
    LSP_HIP(hipStreamSynchronize(stream));
    for (auto it = pool.begin(); it != pool.end();) {
        if (it->first.compare(0, prefix.size(), prefix) == 0) {
            if (it->second.p) LSP_HIP(hipFree(it->second.p));
            it = pool.erase(it);
        } else {
            ++it;
        }
    }
}

void* lsp_ctx::hbuf(const std::string& name, size_t bytes, unsigned flags) {
    Buf& b = hpool[name];
    if (b.cap < bytes) {
        if (b.p) {
            LSP_HIP(hipStreamSynchronize(stream));
            LSP_HIP(hipHostFree(b.p));
            b.p = nullptr;
            b.cap = 0;
        }
        if (bytes) {
            if (hipHostMalloc(&b.p, bytes, flags ? flags : hipHostMallocDefault) != hipSuccess) {
                (void)hipGetLastError();
                throw lsp::LspError(LSP_E_OOM, "hipHostMalloc(" + std::to_string(bytes) + ") for " + name + " failed");
            }
            b.cap = bytes;
        }
    }
    return b.p;
}

void lsp_ctx::h2d_async(const std::string& name, void* dst, const void* src, size_t bytes) {
    if (!bytes) return;
    auto it = stage_ev.find(name);
    if (it == stage_ev.end()) {
        hipEvent_t ev;
        LSP_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        it = stage_ev.emplace(name, ev).first;
    } else {
        LSP_HIP(hipEventSynchronize(it->second));
    }
    void* h = hbuf(name, bytes);
    std::memcpy(h, src, bytes);
    LSP_HIP(hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, stream));
    LSP_HIP(hipEventRecord(it->second, stream));
}

hipStream_t lsp_ctx::side() {
    if (!side_stream) {
        int least = 0, greatest = 0;
        LSP_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        LSP_HIP(hipStreamCreateWithPriority(&side_stream, hipStreamNonBlocking, least));
        LSP_HIP(hipEventCreateWithFlags(&ev_wide, hipEventDisableTiming));
        LSP_HIP(hipEventCreateWithFlags(&ev_side, hipEventDisableTiming));
    }
    return side_stream;
}

lsp::HostPool& lsp_ctx::host_pool() {
    if (!pool_) {
        pool_.reset(new lsp::HostPool(lsp::default_host_threads() - 1));
    }
    return *pool_;
}

// The host pool's size: up to 16 threads (a 1-GPU box's CPU share).  The CPUs
// counted are this process's affinity set (hardware_concurrency() counts the
// whole machine: 256 on a box whose GPU share is 16).  When the launcher says
// several ranks share this host (torchrun's LOCAL_WORLD_SIZE), the set is
// divided among them: the library cannot tell a set the ranks share from a
// slice a launcher pinned for this rank alone, and of the two mistakes
// dividing a private slice only makes the pool smaller, while not dividing a
// shared one puts ranks x 16 spinning threads on it.  The Python
// launch path (replicas.init_from_env) compares the ranks' sets and exports
// the exact size as LSP_HOST_THREADS, which overrides this; other launchers
// that pin each rank to its own CPUs set LSP_HOST_THREADS themselves (lsp.h).
unsigned lsp::default_host_threads() {
    unsigned ranks = 1;
    if (const char* e = std::getenv("LOCAL_WORLD_SIZE")) ranks = (unsigned)std::max(1L, std::strtol(e, nullptr, 10));
    unsigned cpus = std::max(1u, std::thread::hardware_concurrency());
#if defined(__linux__)
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) cpus = (unsigned)CPU_COUNT(&set);
#endif
    unsigned n = std::min(16u, std::max(1u, cpus / ranks));
    if (const char* e = std::getenv("LSP_HOST_THREADS")) n = (unsigned)std::max(1L, std::strtol(e, nullptr, 10));
    return n;
}

const uint4* lsp_ctx::twiddle29(uint32_t logH, bool inverse) {
    using namespace lsp;
    auto key = std::make_pair(logH, inverse ? 1 : 0);
    auto it = twiddles.find(key);
    if (it != twiddles.end()) return it->second;
    const size_t half = logH ? (size_t(1) << (logH - 1)) : 1;
    Fr w = host_two_adic_generator(logH);
    if (inverse) w = fr_inv(w);
    const uint32_t lg = logH ? logH - 1 : 0;
    const uint32_t L1 = (lg + 1) / 2, L2 = lg - L1;
    Fr* tab = fbuf("tw_tab_tmp", (1ull << L1) + (1ull << L2));
    Fr* base = fbuf("tw_base_tmp", 1);
    LSP_HIP(hipMemcpyAsync(base, &w, sizeof(Fr), hipMemcpyHostToDevice, stream));
    LSP_HIP(launch_pow_tables(base, 1, L1, L2, nullptr, tab, stream));
    Fr* pw = fbuf("tw_pow_tmp", half);
    LSP_HIP(launch_powers(tab, L1, half, pw, stream));
    uint4* out = nullptr;
    const size_t n = logH ? (size_t(1) << logH) - 1 : 1;
    LSP_HIP(hipMalloc(&out, n * 3 * sizeof(uint4)));
    LSP_HIP(launch_stage_twiddles(pw, logH, out, stream));
    LSP_HIP(hipStreamSynchronize(stream));
    twiddles[key] = out;
    return out;
}

void lsp_ctx::sync() { LSP_HIP(hipStreamSynchronize(stream)); }
