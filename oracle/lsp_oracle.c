/*
 * lsp_oracle.c -- plain-C restatement of the reference prover's hot path.
 * TEST INFRASTRUCTURE ONLY (checker + timed CPU baseline); see lsp_oracle.h.
 *
 * Reference map (paths relative to the reference repo; [EXT] = the Plonky3
 * fork distributed-lab/Plonky3@f888f90, Cargo.lock:505-711, not vendored):
 *   field            ark-ff 0.5 Montgomery Fr (Cargo.lock:83), bin/src/config.rs:9
 *   coset LDE        [EXT p3-dft] Radix2DitParallel::coset_lde_batch, bin/src/config.rs:22
 *   Poseidon2        [EXT p3-poseidon2] Perm::new_from_rng(8,22), bin/src/main.rs:49
 *   sponge/compress  [EXT p3-symmetric] bin/src/config.rs:12,17
 *   Merkle           [EXT p3-merkle-tree] bin/src/config.rs:19-20
 *   quotient         [EXT p3-uni-stark quotient_values] + air/src/lib.rs:57-167
 *   open / FRI       [EXT p3-fri] TwoAdicFriPcs::open, commit_phase, fold_matrix
 *   transcript       [EXT p3-challenger] HashChallenger, bin/src/config.rs:23
 *   prove/verify     [EXT p3-uni-stark] bin/src/main.rs:80-96
 *   witness          trace/src/permutation.rs:24-93
 */
#include "lsp_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------ field */
static const uint64_t MOD[4] = {0x0a11800000000001ULL, 0x59aa76fed0000001ULL,
                                0x60b44d1e5c37b001ULL, 0x12ab655e9a2ca556ULL};
static const uint64_t MINV = 0x0a117fffffffffffULL; /* -MOD^-1 mod 2^64 */
/* R^2 mod MOD, R = 2^256 */
static uint64_t R2[4];
static lo_fr ONE, ZERO_FR;
static int field_ready = 0;

static int geq_mod(const uint64_t a[4]) {
    for (int i = 3; i >= 0; --i) {
        if (a[i] > MOD[i]) return 1;
        if (a[i] < MOD[i]) return 0;
    }
    return 1;
}

static void sub_mod_raw(uint64_t a[4]) {
    uint64_t borrow = 0;
    for (int i = 0; i < 4; ++i) {
        u128 d = (u128)a[i] - MOD[i] - borrow;
        a[i] = (uint64_t)d;
        borrow = (uint64_t)(d >> 64) ? 1 : 0;
    }
}

static inline void fadd(const lo_fr *a, const lo_fr *b, lo_fr *o) {
    uint64_t c = 0, r[4];
    for (int i = 0; i < 4; ++i) {
        u128 s = (u128)a->l[i] + b->l[i] + c;
        r[i] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
    }
    if (geq_mod(r)) sub_mod_raw(r);
    memcpy(o->l, r, 32);
}

static inline void fsub(const lo_fr *a, const lo_fr *b, lo_fr *o) {
    uint64_t borrow = 0, r[4];
    for (int i = 0; i < 4; ++i) {
        u128 d = (u128)a->l[i] - b->l[i] - borrow;
        r[i] = (uint64_t)d;
        borrow = (uint64_t)(d >> 64) ? 1 : 0;
    }
    if (borrow) {
        uint64_t c = 0;
        for (int i = 0; i < 4; ++i) {
            u128 s = (u128)r[i] + MOD[i] + c;
            r[i] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
    }
    memcpy(o->l, r, 32);
}

static inline void fmul(const lo_fr *a, const lo_fr *b, lo_fr *o) {
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
        uint64_t c = 0;
        for (int j = 0; j < 4; ++j) {
            u128 x = (u128)a->l[j] * b->l[i] + t[j] + c;
            t[j] = (uint64_t)x;
            c = (uint64_t)(x >> 64);
        }
        u128 x = (u128)t[4] + c;
        t[4] = (uint64_t)x;
        t[5] = (uint64_t)(x >> 64);
        uint64_t m = t[0] * MINV;
        x = (u128)m * MOD[0] + t[0];
        c = (uint64_t)(x >> 64);
        for (int j = 1; j < 4; ++j) {
            x = (u128)m * MOD[j] + t[j] + c;
            t[j - 1] = (uint64_t)x;
            c = (uint64_t)(x >> 64);
        }
        x = (u128)t[4] + c;
        t[3] = (uint64_t)x;
        t[4] = t[5] + (uint64_t)(x >> 64);
    }
    uint64_t r[4] = {t[0], t[1], t[2], t[3]};
    if (t[4] || geq_mod(r)) sub_mod_raw(r);
    memcpy(o->l, r, 32);
}

static int fis_zero(const lo_fr *a) { return !(a->l[0] | a->l[1] | a->l[2] | a->l[3]); }
static int feq(const lo_fr *a, const lo_fr *b) { return !memcmp(a->l, b->l, 32); }

static void field_init(void) {
    if (field_ready) return;
    /* R mod MOD by repeated doubling of 1 (2^256 mod MOD), then R^2 = R*R
     * computed by 256 more doublings of R */
    uint64_t x[4] = {1, 0, 0, 0};
    for (int k = 0; k < 512; ++k) {
        uint64_t c = 0;
        for (int i = 0; i < 4; ++i) {
            uint64_t nc = x[i] >> 63;
            x[i] = (x[i] << 1) | c;
            c = nc;
        }
        if (c || geq_mod(x)) sub_mod_raw(x);
        if (k == 255) memcpy(ONE.l, x, 32); /* R mod MOD = Montgomery one */
    }
    memcpy(R2, x, 32);
    memset(&ZERO_FR, 0, sizeof ZERO_FR);
    field_ready = 1;
}

void lo_fr_from_canonical(const uint64_t in[4], lo_fr *out) {
    field_init();
    lo_fr a, r2;
    memcpy(a.l, in, 32);
    memcpy(r2.l, R2, 32);
    fmul(&a, &r2, out);
}

void lo_fr_to_canonical(const lo_fr *a, uint64_t out[4]) {
    field_init();
    lo_fr one = {{1, 0, 0, 0}}, r;
    fmul(a, &one, &r);
    memcpy(out, r.l, 32);
}

void lo_fr_from_u64(uint64_t x, lo_fr *out) {
    uint64_t c[4] = {x, 0, 0, 0};
    lo_fr_from_canonical(c, out);
}

static lo_fr fu(uint64_t x) {
    lo_fr r;
    lo_fr_from_u64(x, &r);
    return r;
}

static void fpow_u(const lo_fr *b, const uint64_t e[4], lo_fr *o) {
    /* left-to-right square-and-multiply from the top set bit */
    lo_fr r = ONE;
    int started = 0;
    for (int i = 3; i >= 0; --i)
        for (int k = 63; k >= 0; --k) {
            if (started) fmul(&r, &r, &r);
            if ((e[i] >> k) & 1) {
                fmul(&r, b, &r);
                started = 1;
            }
        }
    *o = r;
}

static void fpow64(const lo_fr *b, uint64_t e, lo_fr *o) {
    uint64_t ee[4] = {e, 0, 0, 0};
    fpow_u(b, ee, o);
}

static void finv(const lo_fr *a, lo_fr *o) {
    uint64_t e[4];
    memcpy(e, MOD, 32);
    e[0] -= 2; /* MOD[0] = ...0001, no borrow */
    fpow_u(a, e, o);
}

void lo_fr_mul(const lo_fr *a, const lo_fr *b, lo_fr *o) { field_init(); fmul(a, b, o); }
void lo_fr_add(const lo_fr *a, const lo_fr *b, lo_fr *o) { field_init(); fadd(a, b, o); }
void lo_fr_inv(const lo_fr *a, lo_fr *o) { field_init(); finv(a, o); }

/* GENERATOR = 22 (U9); two-adic generator of order 2^bits */
static lo_fr GEN;
static lo_fr two_adic_gen(uint32_t bits) {
    /* ROOT_2_47 = 22^((MOD-1)>>47) */
    uint64_t e[4];
    memcpy(e, MOD, 32);
    e[0] -= 1;
    for (int k = 0; k < 47; ++k) { /* shift right by 47 */
        e[0] = (e[0] >> 1) | (e[1] << 63);
        e[1] = (e[1] >> 1) | (e[2] << 63);
        e[2] = (e[2] >> 1) | (e[3] << 63);
        e[3] >>= 1;
    }
    lo_fr g = fu(22), r;
    fpow_u(&g, e, &r);
    for (uint32_t k = bits; k < 47; ++k) fmul(&r, &r, &r);
    return r;
}

static uint64_t bitrev64(uint64_t x, uint32_t bits) {
    uint64_t r = 0;
    for (uint32_t i = 0; i < bits; ++i) {
        r = (r << 1) | (x & 1);
        x >>= 1;
    }
    return r;
}

static uint32_t log2_strict(size_t n) {
    uint32_t b = 0;
    while (((size_t)1 << b) < n) ++b;
    return ((size_t)1 << b) == n ? b : 0xFFFFFFFFu;
}

/* ------------------------------------------------------------ phase timer */
/* LO_TIME=1: lo_prove prints each phase's wall time to stderr (profiling the
 * checker itself; off by default) */
#include <stdio.h>
#include <time.h>
static double lo_now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}
static void lo_phase(const char *name, double *t0) {
    static int on = -1;
    if (on < 0) on = getenv("LO_TIME") != NULL;
    if (!on) return;
    double t = lo_now();
    fprintf(stderr, "[oracle] %-28s %8.3f s\n", name, t - *t0);
    *t0 = t;
}

/* ---------------------------------------------------------------- threads */
typedef void (*range_fn)(void *ctx, size_t lo, size_t hi);
typedef struct { range_fn fn; void *ctx; size_t lo, hi; } job_t;
static void *job_run(void *a) {
    job_t *j = (job_t *)a;
    j->fn(j->ctx, j->lo, j->hi);
    return NULL;
}
static void parallel_for(size_t n, int nthreads, range_fn fn, void *ctx) {
    if (nthreads <= 1 || n < 64) {
        fn(ctx, 0, n);
        return;
    }
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    job_t jobs[256];
    size_t chunk = (n + nthreads - 1) / nthreads;
    int used = 0;
    for (int t = 0; t < nthreads; ++t) {
        size_t lo = (size_t)t * chunk, hi = lo + chunk > n ? n : lo + chunk;
        if (lo >= hi) break;
        jobs[t] = (job_t){fn, ctx, lo, hi};
        pthread_create(&th[t], NULL, job_run, &jobs[t]);
        used++;
    }
    for (int t = 0; t < used; ++t) pthread_join(th[t], NULL);
}

/* batch inverse (Montgomery trick) in parallel chunks */
typedef struct { const lo_fr *in; lo_fr *out; } binv_ctx;
static void binv_range(void *c, size_t lo, size_t hi) {
    binv_ctx *b = (binv_ctx *)c;
    if (lo >= hi) return;
    lo_fr acc = ONE;
    for (size_t i = lo; i < hi; ++i) {
        b->out[i] = acc;
        fmul(&acc, &b->in[i], &acc);
    }
    lo_fr inv;
    finv(&acc, &inv);
    for (size_t i = hi; i-- > lo;) {
        lo_fr t;
        fmul(&inv, &b->out[i], &t);
        fmul(&inv, &b->in[i], &inv);
        b->out[i] = t;
    }
}
static void batch_inverse(const lo_fr *in, lo_fr *out, size_t n, int nthreads) {
    binv_ctx c = {in, out};
    parallel_for(n, nthreads, binv_range, &c);
}

/* ------------------------------------------------------------ SplitMix64 */
typedef struct { uint64_t s; } smix;
static uint64_t smix_next(smix *r) {
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static lo_fr smix_fr(smix *r) {
    for (;;) {
        uint64_t v[4];
        for (int k = 0; k < 4; ++k) v[k] = smix_next(r);
        v[3] &= (1ULL << 61) - 1; /* 253 bits */
        if (!geq_mod(v)) {
            lo_fr o;
            lo_fr_from_canonical(v, &o);
            return o;
        }
    }
}
static uint64_t smix_below(smix *r, uint64_t n) {
    /* same rule as pyoracle.SplitMix64.below: accept x < 2^64 - (2^64 mod n) */
    u128 two64 = (u128)1 << 64;
    u128 lim = two64 - (two64 % n);
    for (;;) {
        uint64_t x = smix_next(r);
        if ((u128)x < lim) return x % n;
    }
}

void lo_setup(uint64_t seed, uint32_t sbox_degree, uint32_t rounds_f, uint32_t rounds_p, lo_params *out) {
    field_init();
    memset(out, 0, sizeof *out);
    smix r = {seed};
    out->sbox_degree = sbox_degree;
    out->rounds_f = rounds_f;
    out->rounds_p = rounds_p;
    out->alpha = smix_fr(&r);
    out->delta = smix_fr(&r);
    for (uint32_t i = 0; i < rounds_f / 2; ++i)
        for (int j = 0; j < 3; ++j) out->ext_initial[i][j] = smix_fr(&r);
    for (uint32_t i = 0; i < rounds_f / 2; ++i)
        for (int j = 0; j < 3; ++j) out->ext_terminal[i][j] = smix_fr(&r);
    for (uint32_t i = 0; i < rounds_p; ++i) out->internal[i] = smix_fr(&r);
}

/* -------------------------------------------------------------- Poseidon2 */
/* x^D (D = sbox_degree: 11, or 17 for the other BLS12-377 instance) by
 * left-to-right square-and-multiply over D's own bits: 3 squares and 2
 * products for D = 11 (fpow64 would walk a 256-bit exponent from the top) */
static inline void sbox(const lo_params *p, lo_fr *x) {
    const uint32_t d = p->sbox_degree;
    const lo_fr b = *x;
    lo_fr r = b;
    for (int k = 30 - __builtin_clz(d); k >= 0; --k) {
        fmul(&r, &r, &r);
        if ((d >> k) & 1) fmul(&r, &b, &r);
    }
    *x = r;
}
/* generic U2/U3 layers (lo_params.generic_lin) */
static void ext_layer_gen(const lo_params *p, lo_fr s[3]) {
    lo_fr o[3];
    for (int i = 0; i < 3; ++i) {
        lo_fr acc = ZERO_FR, t;
        for (int j = 0; j < 3; ++j) {
            fmul(&p->ext_mds[3 * i + j], &s[j], &t);
            fadd(&acc, &t, &acc);
        }
        o[i] = acc;
    }
    for (int i = 0; i < 3; ++i) s[i] = o[i];
}
static void int_layer_gen(const lo_params *p, lo_fr s[3]) {
    lo_fr u, t;
    fadd(&s[0], &s[1], &u);
    fadd(&u, &s[2], &u);
    for (int i = 0; i < 3; ++i) {
        fmul(&p->int_diag[i], &s[i], &t);
        fadd(&u, &t, &s[i]);
    }
}
static inline void ext_layer(lo_fr s[3]) {
    lo_fr t;
    fadd(&s[0], &s[1], &t);
    fadd(&t, &s[2], &t);
    fadd(&s[0], &t, &s[0]);
    fadd(&s[1], &t, &s[1]);
    fadd(&s[2], &t, &s[2]);
}
static inline void int_layer(lo_fr s[3]) {
    lo_fr t;
    fadd(&s[0], &s[1], &t);
    fadd(&t, &s[2], &t);
    fadd(&s[0], &t, &s[0]);
    fadd(&s[1], &t, &s[1]);
    fadd(&s[2], &s[2], &s[2]);
    fadd(&s[2], &t, &s[2]);
}
void lo_poseidon2_permute(const lo_params *p, lo_fr s[3]) {
    field_init();
    const int gen = p->generic_lin != 0;
#define EXT() (gen ? ext_layer_gen(p, s) : ext_layer(s))
    EXT();
    for (uint32_t r = 0; r < p->rounds_f / 2; ++r) {
        for (int i = 0; i < 3; ++i) {
            fadd(&s[i], &p->ext_initial[r][i], &s[i]);
            sbox(p, &s[i]);
        }
        EXT();
    }
    for (uint32_t r = 0; r < p->rounds_p; ++r) {
        fadd(&s[0], &p->internal[r], &s[0]);
        sbox(p, &s[0]);
        if (gen)
            int_layer_gen(p, s);
        else
            int_layer(s);
    }
    for (uint32_t r = 0; r < p->rounds_f / 2; ++r) {
        for (int i = 0; i < 3; ++i) {
            fadd(&s[i], &p->ext_terminal[r][i], &s[i]);
            sbox(p, &s[i]);
        }
        EXT();
    }
#undef EXT
}

/* PaddingFreeSponge<Perm,3,2,1>: overwrite-mode, no padding */
void lo_hash_iter(const lo_params *p, const lo_fr *in, size_t n, lo_fr *out) {
    lo_fr s[3] = {ZERO_FR, ZERO_FR, ZERO_FR};
    field_init();
    size_t pos = 0;
    for (;;) {
        for (int i = 0; i < 2; ++i) {
            if (pos < n) {
                s[i] = in[pos++];
            } else {
                if (i != 0) lo_poseidon2_permute(p, s);
                *out = s[0];
                return;
            }
        }
        lo_poseidon2_permute(p, s);
    }
}
static void compress2(const lo_params *p, const lo_fr *l, const lo_fr *r, lo_fr *o) {
    lo_fr s[3] = {*l, *r, ZERO_FR};
    lo_poseidon2_permute(p, s);
    *o = s[0];
}

/* ------------------------------------------------------------------ Merkle */
typedef struct { const lo_params *p; const lo_fr *rows; size_t W; lo_fr *dst; const lo_fr *src; } mk_ctx;
static void mk_leaves(void *c, size_t lo, size_t hi) {
    mk_ctx *m = (mk_ctx *)c;
    for (size_t i = lo; i < hi; ++i) lo_hash_iter(m->p, m->rows + i * m->W, m->W, &m->dst[i]);
}
static void mk_level(void *c, size_t lo, size_t hi) {
    mk_ctx *m = (mk_ctx *)c;
    for (size_t i = lo; i < hi; ++i) compress2(m->p, &m->src[2 * i], &m->src[2 * i + 1], &m->dst[i]);
}
void lo_merkle_commit(const lo_params *p, const lo_fr *rows, size_t h, size_t W, lo_fr *layers, int nthreads) {
    field_init();
    mk_ctx c = {p, rows, W, layers, NULL};
    parallel_for(h, nthreads, mk_leaves, &c);
    size_t off = 0, len = h;
    while (len > 1) {
        c.src = layers + off;
        c.dst = layers + off + len;
        parallel_for(len / 2, nthreads, mk_level, &c);
        off += len;
        len /= 2;
    }
}

/* ------------------------------------------------------------------- NTT */
/* natural-order in-place DFT with root w (order n): bit-reversal, then
 * radix-2 DIT stages.  With nthreads > 1 each stage's n/2 butterflies (and the
 * bit-reversal) are split over threads -- the same butterflies, the same
 * twiddles, so the same result bits for any thread count. */
typedef struct { lo_fr *a; size_t n, half; uint32_t lg; lo_fr wl; } ntt_ctx;
static void ntt_bitrev_range(void *c, size_t lo, size_t hi) {
    ntt_ctx *t = (ntt_ctx *)c;
    for (size_t i = lo; i < hi; ++i) {
        size_t j = (size_t)bitrev64(i, t->lg);
        if (j > i) { /* the pair belongs to the range holding i */
            lo_fr x = t->a[i];
            t->a[i] = t->a[j];
            t->a[j] = x;
        }
    }
}
static void ntt_stage_range(void *c, size_t lo, size_t hi) {
    /* butterflies k in [lo, hi): block k / half, offset j = k % half */
    ntt_ctx *t = (ntt_ctx *)c;
    size_t half = t->half, j = lo % half;
    lo_fr w;
    fpow64(&t->wl, j, &w);
    for (size_t k = lo; k < hi; ++k) {
        size_t i = (k / half) * 2 * half + j;
        lo_fr u = t->a[i], v;
        fmul(&t->a[i + half], &w, &v);
        fadd(&u, &v, &t->a[i]);
        fsub(&u, &v, &t->a[i + half]);
        if (++j == half) {
            j = 0;
            w = ONE;
        } else {
            fmul(&w, &t->wl, &w);
        }
    }
}
static void ntt_inplace_mt(lo_fr *a, size_t n, const lo_fr *root, int nthreads) {
    ntt_ctx c = {a, n, 0, log2_strict(n), ONE};
    parallel_for(n, nthreads, ntt_bitrev_range, &c);
    for (size_t len = 2; len <= n; len <<= 1) {
        fpow64(root, n / len, &c.wl);
        c.half = len / 2;
        parallel_for(n / 2, nthreads, ntt_stage_range, &c);
    }
}
static void ntt_inplace(lo_fr *a, size_t n, const lo_fr *root) { ntt_inplace_mt(a, n, root, 1); }

typedef struct {
    const lo_fr *in; size_t h, w; uint32_t added; const lo_fr *shifts; lo_fr *out;
    int ntt_threads; /* threads inside each column's NTTs (1: columns run in parallel instead) */
} lde_ctx;
/* coefficient i of column col times shift^i / h, and the zero padding */
typedef struct { lo_fr *buf; size_t h, N; lo_fr hinv, shift; } twist_ctx;
static void twist_range(void *c, size_t lo, size_t hi) {
    twist_ctx *t = (twist_ctx *)c;
    lo_fr s;
    fpow64(&t->shift, lo, &s);
    fmul(&s, &t->hinv, &s);
    for (size_t i = lo; i < hi; ++i) {
        if (i < t->h) {
            fmul(&t->buf[i], &s, &t->buf[i]);
            fmul(&s, &t->shift, &s);
        } else {
            t->buf[i] = ZERO_FR;
        }
    }
}
/* output row i of column col = buf[bitrev(i)] (the bit-reversed LDE) */
typedef struct { const lo_fr *buf; lo_fr *out; size_t w, col; uint32_t lgN; } scatter_ctx;
static void scatter_range(void *c, size_t lo, size_t hi) {
    scatter_ctx *t = (scatter_ctx *)c;
    for (size_t i = lo; i < hi; ++i) t->out[i * t->w + t->col] = t->buf[bitrev64(i, t->lgN)];
}
static void lde_cols(void *c, size_t lo, size_t hi) {
    lde_ctx *L = (lde_ctx *)c;
    size_t h = L->h, N = h << L->added;
    uint32_t lgN = log2_strict(N);
    lo_fr *buf = (lo_fr *)malloc(N * sizeof(lo_fr));
    lo_fr wh_inv, wN, hinv;
    lo_fr wh = two_adic_gen(log2_strict(h));
    finv(&wh, &wh_inv);
    wN = two_adic_gen(lgN);
    lo_fr hf = fu(h);
    finv(&hf, &hinv);
    for (size_t col = lo; col < hi; ++col) {
        for (size_t i = 0; i < h; ++i) buf[i] = L->in[i * L->w + col];
        ntt_inplace_mt(buf, h, &wh_inv, L->ntt_threads); /* h * coefficients */
        twist_ctx tc = {buf, h, N, hinv, L->shifts[col]};  /* shift^i / h, then zeros */
        parallel_for(N, L->ntt_threads, twist_range, &tc);
        ntt_inplace_mt(buf, N, &wN, L->ntt_threads);
        scatter_ctx sc = {buf, L->out, L->w, col, lgN};
        parallel_for(N, L->ntt_threads, scatter_range, &sc);
    }
    free(buf);
}
/* Columns in parallel when there are at least as many as threads (or the
 * transform is small); otherwise one column at a time with each NTT stage
 * split over the threads (the quotient's 4 chunks, the 3x3 trace's 8 columns
 * on 16 threads). */
void lo_coset_lde_batch(const lo_fr *in, size_t h, size_t w, uint32_t added_bits,
                        const lo_fr *shifts, lo_fr *out, int nthreads) {
    field_init();
    lde_ctx c = {in, h, w, added_bits, shifts, out, 1};
    if (nthreads > 1 && (size_t)nthreads > w && (h << added_bits) >= ((size_t)1 << 14)) {
        c.ntt_threads = nthreads;
        lde_cols(&c, 0, w);
        return;
    }
    if (nthreads <= 1 || w < 2) {
        lde_cols(&c, 0, w);
        return;
    }
    pthread_t th[256];
    job_t jobs[256];
    size_t chunk = (w + nthreads - 1) / nthreads;
    int used = 0;
    for (int t = 0; t < nthreads; ++t) {
        size_t lo = t * chunk, hi = lo + chunk > w ? w : lo + chunk;
        if (lo >= hi) break;
        jobs[t] = (job_t){lde_cols, &c, lo, hi};
        pthread_create(&th[t], NULL, job_run, &jobs[t]);
        used++;
    }
    for (int t = 0; t < used; ++t) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------ point evaluation */
/* Barycentric evaluation of the columns given on H_h, independent of any NTT:
 * p(x) = (x^h - 1)/h * sum_i y_i w^i / (x - w^i).  The full-size LDE checks
 * (tests/test_gpu_fullsize.py) use it where the oracle's own LDE would take
 * minutes.  Work is split into blocks of rows; each block inverts its own
 * denominators and keeps a partial sum per column. */
typedef struct {
    const lo_fr *in; size_t h, w, nblk; lo_fr x, wh; lo_fr *part;
} ev_ctx;
static void ev_blocks(void *c, size_t lo, size_t hi) {
    ev_ctx *E = (ev_ctx *)c;
    for (size_t b = lo; b < hi; ++b) {
        size_t r0 = b * E->h / E->nblk, r1 = (b + 1) * E->h / E->nblk, n = r1 - r0;
        lo_fr *wi = (lo_fr *)malloc(n * sizeof(lo_fr)), *den = (lo_fr *)malloc(n * sizeof(lo_fr));
        lo_fr *inv = (lo_fr *)malloc(n * sizeof(lo_fr));
        lo_fr cur;
        fpow64(&E->wh, r0, &cur);
        for (size_t i = 0; i < n; ++i) {
            wi[i] = cur;
            fsub(&E->x, &cur, &den[i]);
            fmul(&cur, &E->wh, &cur);
        }
        binv_ctx bc = {den, inv};
        binv_range(&bc, 0, n);
        lo_fr *acc = E->part + b * E->w;
        for (size_t c2 = 0; c2 < E->w; ++c2) acc[c2] = ZERO_FR;
        for (size_t i = 0; i < n; ++i) {
            lo_fr f, t;
            fmul(&wi[i], &inv[i], &f);
            for (size_t c2 = 0; c2 < E->w; ++c2) {
                fmul(&E->in[(r0 + i) * E->w + c2], &f, &t);
                fadd(&acc[c2], &t, &acc[c2]);
            }
        }
        free(wi);
        free(den);
        free(inv);
    }
}

void lo_eval_points(const lo_fr *in, size_t h, size_t w, const lo_fr *xs, size_t npts, lo_fr *out, int nthreads) {
    field_init();
    size_t nblk = h < 256 ? h : 256;
    lo_fr *part = (lo_fr *)malloc(nblk * w * sizeof(lo_fr));
    lo_fr hinv, hf = fu(h);
    finv(&hf, &hinv);
    for (size_t k = 0; k < npts; ++k) {
        ev_ctx E = {in, h, w, nblk, xs[k], two_adic_gen(log2_strict(h)), part};
        parallel_for(nblk, nthreads, ev_blocks, &E);
        lo_fr scale; /* (x^h - 1) / h */
        fpow64(&xs[k], h, &scale);
        fsub(&scale, &ONE, &scale);
        fmul(&scale, &hinv, &scale);
        for (size_t c2 = 0; c2 < w; ++c2) {
            lo_fr s = ZERO_FR;
            for (size_t b = 0; b < nblk; ++b) fadd(&s, &part[b * w + c2], &s);
            fmul(&s, &scale, &out[k * w + c2]);
        }
    }
    free(part);
}

/* x_j of LDE output row j (bit-reversed order over N = h << added_bits) */
void lo_lde_point(size_t h, uint32_t added_bits, const lo_fr *shift, uint64_t j, lo_fr *out) {
    field_init();
    uint32_t lgN = log2_strict(h) + added_bits;
    lo_fr wN = two_adic_gen(lgN);
    fpow64(&wN, bitrev64(j, lgN), out);
    fmul(out, shift, out);
}

/* -------------------------------------------------------------------- AIR */
#define MAXC 4096
#define MAXT 32
#define MAXCFG 64
typedef struct {
    int type; /* 1 perm, 2 lookup */
    int na, nb, a[MAXC], b[MAXC], binv, check;
    int ntab, nbc, bt[MAXT][MAXC / 4], a_filter, b_filter[MAXT], a_inv, b_inv[MAXT], occ[MAXT];
} cfg_t;

static int parse_air(const int32_t *air, size_t len, cfg_t *cfgs, int *ncfg) {
    size_t p = 0;
    if (len < 1) return -1;
    int n = air[p++];
    if (n < 1 || n > MAXCFG) return -1;
#define NEXT() (p < len ? air[p++] : (int32_t)-1)
    for (int c = 0; c < n; ++c) {
        cfg_t *g = &cfgs[c];
        memset(g, 0, sizeof *g);
        g->type = NEXT();
        if (g->type == 1) {
            g->na = NEXT();
            g->nb = NEXT();
            if (g->na < 1 || g->na > MAXC || g->nb < 1 || g->nb > MAXC) return -1;
            for (int i = 0; i < g->na; ++i) g->a[i] = NEXT();
            for (int i = 0; i < g->nb; ++i) g->b[i] = NEXT();
            g->binv = NEXT();
            g->check = NEXT();
        } else if (g->type == 2) {
            g->na = NEXT();
            if (g->na < 1 || g->na > MAXC) return -1;
            for (int i = 0; i < g->na; ++i) g->a[i] = NEXT();
            g->ntab = NEXT();
            g->nbc = NEXT();
            if (g->ntab < 1 || g->ntab > MAXT || g->nbc < 1 || g->nbc > MAXC / 4) return -1;
            for (int t = 0; t < g->ntab; ++t)
                for (int i = 0; i < g->nbc; ++i) g->bt[t][i] = NEXT();
            g->a_filter = NEXT();
            for (int t = 0; t < g->ntab; ++t) g->b_filter[t] = NEXT();
            g->a_inv = NEXT();
            for (int t = 0; t < g->ntab; ++t) g->b_inv[t] = NEXT();
            for (int t = 0; t < g->ntab; ++t) g->occ[t] = NEXT();
            g->check = NEXT();
        } else {
            return -1;
        }
    }
#undef NEXT
    if (p != len) return -1;
    *ncfg = n;
    return 0;
}

static int horner_deg(int n, int pd) {
    int d = 0;
    for (int i = 0; i < n; ++i) d = (d + pd) > 1 ? d + pd : 1;
    return d;
}
static int imax(int a, int b) { return a > b ? a : b; }

static int constraint_stats(const cfg_t *cfgs, int n, int pd, int *count) {
    int maxd = 0, k = 0;
    for (int c = 0; c < n; ++c) {
        const cfg_t *g = &cfgs[c];
        if (g->type == 1) {
            int a = imax(horner_deg(g->na, pd), pd), b = imax(horner_deg(g->nb, pd), pd);
            maxd = imax(maxd, b + 1);
            maxd = imax(maxd, 1 + imax(1, a + 1));
            maxd = imax(maxd, imax(1, a + 2));
            maxd = imax(maxd, 2);
            k += 4;
        } else {
            int a = imax(horner_deg(g->na, pd), pd);
            maxd = imax(maxd, a + 1);
            int lc = 2;
            for (int t = 0; t < g->ntab; ++t) {
                maxd = imax(maxd, imax(horner_deg(g->nbc, pd), pd) + 1);
                lc = 3;
            }
            maxd = imax(maxd, 1 + lc);
            maxd = imax(maxd, lc);
            maxd = imax(maxd, 2);
            k += 1 + g->ntab + 3;
        }
    }
    *count = k;
    return maxd;
}

int lo_log_quotient_degree(const int32_t *air, size_t air_len, int public_degree) {
    static cfg_t cfgs[MAXCFG];
    int n, k;
    if (parse_air(air, air_len, cfgs, &n)) return -1;
    int d = constraint_stats(cfgs, n, public_degree, &k);
    if (d < 2) d = 2;
    int lg = 0;
    while ((1 << lg) < d - 1) ++lg;
    return lg;
}

static lo_fr horner(const lo_fr *row, const int *ids, int n, const lo_fr *alpha) {
    lo_fr acc = ZERO_FR;
    for (int i = 0; i < n; ++i) {
        fmul(&acc, alpha, &acc);
        fadd(&acc, &row[ids[i]], &acc);
    }
    return acc;
}

/* folds all constraints of all configs into acc (Horner in alpha), eval order */
static void eval_fold(const cfg_t *cfgs, int n, const lo_fr *loc, const lo_fr *nxt, const lo_fr *ap,
                      const lo_fr *dl, const lo_fr *first, const lo_fr *last, const lo_fr *trans,
                      const lo_fr *alpha, lo_fr *acc) {
#define PUSH(x) do { fmul(acc, alpha, acc); fadd(acc, (x), acc); } while (0)
    for (int c = 0; c < n; ++c) {
        const cfg_t *g = &cfgs[c];
        lo_fr t, u, v;
        if (g->type == 1) {
            lo_fr al = horner(loc, g->a, g->na, ap), bl = horner(loc, g->b, g->nb, ap);
            fadd(&al, dl, &al);
            fadd(&bl, dl, &bl);
            fmul(&bl, &loc[g->binv], &t);
            fsub(&t, &ONE, &t);
            PUSH(&t);
            fmul(&al, &loc[g->binv], &t);
            fsub(&loc[g->check], &t, &t);
            fmul(first, &t, &t);
            PUSH(&t);
            lo_fr an = horner(nxt, g->a, g->na, ap);
            fadd(&an, dl, &an);
            fmul(&loc[g->check], &an, &t);
            fmul(&t, &nxt[g->binv], &t);
            fsub(&nxt[g->check], &t, &t);
            fmul(trans, &t, &t);
            PUSH(&t);
            fsub(&loc[g->check], &ONE, &t);
            fmul(last, &t, &t);
            PUSH(&t);
        } else {
            lo_fr al = horner(loc, g->a, g->na, ap);
            fadd(&al, dl, &al);
            fmul(&al, &loc[g->a_inv], &t);
            fsub(&t, &ONE, &t);
            PUSH(&t);
            lo_fr lc, nc;
            fmul(&loc[g->a_filter], &loc[g->a_inv], &lc);
            fmul(&nxt[g->a_filter], &nxt[g->a_inv], &nc);
            for (int tb = 0; tb < g->ntab; ++tb) {
                lo_fr bl = horner(loc, g->bt[tb], g->nbc, ap);
                fadd(&bl, dl, &bl);
                fmul(&bl, &loc[g->b_inv[tb]], &t);
                fsub(&t, &ONE, &t);
                PUSH(&t);
                fmul(&loc[g->b_filter[tb]], &loc[g->occ[tb]], &u);
                fmul(&u, &loc[g->b_inv[tb]], &u);
                fsub(&lc, &u, &lc);
                fmul(&nxt[g->b_filter[tb]], &nxt[g->occ[tb]], &v);
                fmul(&v, &nxt[g->b_inv[tb]], &v);
                fsub(&nc, &v, &nc);
            }
            fsub(&loc[g->check], &lc, &t);
            fmul(first, &t, &t);
            PUSH(&t);
            fsub(&nxt[g->check], &loc[g->check], &t);
            fsub(&t, &nc, &t);
            fmul(trans, &t, &t);
            PUSH(&t);
            fmul(last, &loc[g->check], &t);
            PUSH(&t);
        }
    }
#undef PUSH
}

/* ------------------------------------------------------------- challenger */
typedef struct {
    const lo_params *p;
    lo_fr in[4096];
    size_t nin;
    lo_fr out[1];
    size_t nout;
    int mont_bits; /* U8: sample_bits from the Montgomery form (LO_T_SAMPLE_BITS_MONT) */
} chal_t;
static void ch_init(chal_t *c, const lo_params *p, uint32_t transcript) {
    c->p = p;
    c->nin = 0;
    c->nout = 0;
    c->mont_bits = (transcript & LO_T_SAMPLE_BITS_MONT) != 0;
}
static void ch_observe(chal_t *c, const lo_fr *x) {
    c->nout = 0;
    if (c->nin < 4096) c->in[c->nin++] = *x;
}
static lo_fr ch_sample(chal_t *c) {
    if (c->nout == 0) {
        lo_fr o;
        lo_hash_iter(c->p, c->in, c->nin, &o);
        c->in[0] = o;
        c->nin = 1;
        c->out[0] = o;
        c->nout = 1;
    }
    return c->out[--c->nout];
}
static uint64_t ch_sample_bits(chal_t *c, uint32_t bits) {
    lo_fr s = ch_sample(c);
    uint64_t can[4];
    if (c->mont_bits)
        memcpy(can, s.l, sizeof can); /* lo_fr holds the reduced Montgomery form */
    else
        lo_fr_to_canonical(&s, can);
    return bits >= 64 ? can[0] : (can[0] & ((1ULL << bits) - 1));
}
static int ch_check_witness(chal_t *c, uint32_t bits, uint64_t w) {
    lo_fr x = fu(w);
    ch_observe(c, &x);
    return ch_sample_bits(c, bits) == 0;
}
static uint64_t ch_grind(chal_t *c, uint32_t bits) {
    for (uint64_t w = 0;; ++w) {
        chal_t probe = *c;
        if (ch_check_witness(&probe, bits, w)) {
            ch_check_witness(c, bits, w);
            return w;
        }
    }
}

/* ------------------------------------------------------------ serializer */
typedef struct { uint8_t *b; size_t n, cap; } buf_t;
static void bput(buf_t *b, const void *d, size_t n) {
    if (b->n + n > b->cap) {
        b->cap = (b->n + n) * 2;
        b->b = (uint8_t *)realloc(b->b, b->cap);
    }
    memcpy(b->b + b->n, d, n);
    b->n += n;
}
static void bput_u32(buf_t *b, uint32_t x) { bput(b, &x, 4); }
static void bput_fr(buf_t *b, const lo_fr *x) {
    uint64_t c[4];
    lo_fr_to_canonical(x, c);
    bput(b, c, 32);
}

/* ------------------------------------------------------------ prover parts */
typedef struct {
    const cfg_t *cfgs; int ncfg; const lo_fr *lde; size_t w; uint32_t logQ, log_q;
    const lo_fr *first, *last, *trans, *invz; const lo_fr *ap, *dl, *alpha; lo_fr *out; size_t Q;
} q_ctx;
static void q_range(void *c, size_t lo, size_t hi) {
    q_ctx *q = (q_ctx *)c;
    size_t step = (size_t)1 << q->log_q;
    for (size_t i = lo; i < hi; ++i) {
        const lo_fr *loc = q->lde + bitrev64(i, q->logQ) * q->w;
        const lo_fr *nxt = q->lde + bitrev64((i + step) % q->Q, q->logQ) * q->w;
        lo_fr acc = ZERO_FR;
        size_t per = (size_t)1 << q->log_q; /* period of Z_H values */
        eval_fold(q->cfgs, q->ncfg, loc, nxt, q->ap, q->dl, &q->first[i], &q->last[i], &q->trans[i],
                  q->alpha, &acc);
        fmul(&acc, &q->invz[i % per], &q->out[i]);
    }
}

typedef struct { lo_fr *a; const lo_fr *sub; lo_fr base; lo_fr mulc; int mode; } vec_ctx;

typedef struct {
    const lo_fr *lde, *qlde; size_t w, q; const lo_fr *invz, *invzn; const lo_fr *apw; /* alpha_fri powers */
    lo_fr ry_z, ry_zn; const lo_fr *ryq; lo_fr *ro;
} red_ctx;
static void red_range(void *c, size_t lo, size_t hi) {
    red_ctx *r = (red_ctx *)c;
    size_t w = r->w, q = r->q;
    for (size_t i = lo; i < hi; ++i) {
        lo_fr rr = ZERO_FR, t, acc = ZERO_FR;
        for (size_t k = 0; k < w; ++k) {
            fmul(&r->apw[k], &r->lde[i * w + k], &t);
            fadd(&rr, &t, &rr);
        }
        /* trace @ zeta: alpha^0 * (ry - rr) * invz */
        fsub(&r->ry_z, &rr, &t);
        fmul(&t, &r->invz[i], &t);
        fadd(&acc, &t, &acc);
        /* trace @ zeta_next: alpha^w */
        fsub(&r->ry_zn, &rr, &t);
        fmul(&t, &r->invzn[i], &t);
        fmul(&t, &r->apw[w], &t);
        fadd(&acc, &t, &acc);
        for (size_t j = 0; j < q; ++j) {
            fsub(&r->ryq[j], &r->qlde[i * q + j], &t);
            fmul(&t, &r->invz[i], &t);
            fmul(&t, &r->apw[2 * w + j], &t);
            fadd(&acc, &t, &acc);
        }
        r->ro[i] = acc;
    }
}

typedef struct { const lo_fr *v; lo_fr *o; lo_fr half, hb; const lo_fr *gpow; uint32_t logm; } fold_ctx;
static void fold_range(void *c, size_t lo, size_t hi) {
    fold_ctx *f = (fold_ctx *)c;
    for (size_t i = lo; i < hi; ++i) {
        lo_fr p, a, b, t;
        fmul(&f->hb, &f->gpow[bitrev64(i, f->logm)], &p);
        fadd(&f->half, &p, &a);
        fsub(&f->half, &p, &b);
        fmul(&a, &f->v[2 * i], &t);
        fmul(&b, &f->v[2 * i + 1], &a);
        fadd(&t, &a, &f->o[i]);
    }
}

typedef struct { lo_fr *dst; lo_fr base; } pow_ctx;
static void pow_range(void *c, size_t lo, size_t hi) {
    pow_ctx *p = (pow_ctx *)c;
    lo_fr x;
    fpow64(&p->base, lo, &x);
    for (size_t i = lo; i < hi; ++i) {
        p->dst[i] = x;
        fmul(&x, &p->base, &x);
    }
}
static void powers(lo_fr base, size_t n, lo_fr *dst, int nthreads) {
    pow_ctx c = {dst, base};
    parallel_for(n, nthreads, pow_range, &c);
}

/* the LDE's points in row order: xs[i] = GEN w_N^bitrev(i) */
typedef struct { const lo_fr *nat; lo_fr *xs; uint32_t logN; } xs_ctx;
static void xs_range(void *c, size_t lo, size_t hi) {
    xs_ctx *x = (xs_ctx *)c;
    for (size_t i = lo; i < hi; ++i) fmul(&GEN, &x->nat[bitrev64(i, x->logN)], &x->xs[i]);
}

typedef struct { const lo_fr *xs; lo_fr z; lo_fr *out; } den_ctx;
static void den_range(void *c, size_t lo, size_t hi) {
    den_ctx *d = (den_ctx *)c;
    for (size_t i = lo; i < hi; ++i) fsub(&d->z, &d->xs[i], &d->out[i]);
}

/* barycentric opened values over the first h rows (bit-reversed low coset):
 * ys[c] = (z^h - g^h)/(g^h h) * sum_i M[i][c] * x_i / (z - x_i) */
static void interpolate(const lo_fr *mat, size_t h, size_t w, const lo_fr *xs, const lo_fr *invd,
                        const lo_fr *z, lo_fr *ys) {
    for (size_t c = 0; c < w; ++c) ys[c] = ZERO_FR;
    for (size_t i = 0; i < h; ++i) {
        lo_fr s;
        fmul(&xs[i], &invd[i], &s);
        for (size_t c = 0; c < w; ++c) {
            lo_fr t;
            fmul(&mat[i * w + c], &s, &t);
            fadd(&ys[c], &t, &ys[c]);
        }
    }
    lo_fr zh, gh, f, t;
    fpow64(z, h, &zh);
    fpow64(&GEN, h, &gh);
    fsub(&zh, &gh, &f);
    lo_fr hh = fu(h);
    fmul(&gh, &hh, &t);
    finv(&t, &t);
    fmul(&f, &t, &f);
    for (size_t c = 0; c < w; ++c) fmul(&ys[c], &f, &ys[c]);
}

static void tree_path(const lo_fr *layers, size_t nleaves, size_t index, buf_t *b) {
    size_t off = 0, len = nleaves;
    uint32_t lg = log2_strict(nleaves);
    bput_u32(b, lg);
    for (uint32_t i = 0; i < lg; ++i) {
        bput_fr(b, &layers[off + ((index >> i) ^ 1)]);
        off += len;
        len >>= 1;
    }
}

void *lo_alloc(size_t bytes) { return malloc(bytes); }
void lo_free(void *ptr) { free(ptr); }

int lo_prove(const lo_params *p, const lo_fri *fri, const lo_fr *trace, size_t h, size_t w,
             const int32_t *air, size_t air_len, int public_degree, int nthreads,
             uint8_t **proof_out, size_t *proof_len, lo_debug *dbg) {
    field_init();
    GEN = fu(22);
    static cfg_t cfgs[MAXCFG];
    int ncfg, K;
    if (parse_air(air, air_len, cfgs, &ncfg)) return -1;
    uint32_t log_h = log2_strict(h);
    if (log_h == 0xFFFFFFFFu || h < 2) return -2;
    int maxd = constraint_stats(cfgs, ncfg, public_degree, &K);
    if (maxd < 2) maxd = 2;
    uint32_t log_q = 0;
    while ((1 << log_q) < maxd - 1) ++log_q;
    size_t q = (size_t)1 << log_q;
    uint32_t lb = fri->log_blowup;
    if (log_q > lb) return -3;
    size_t N = h << lb, Q = h << log_q;
    uint32_t logN = log_h + lb, logQ = log_h + log_q;

    double tph = lo_now();
    /* ---- commit to trace data */
    lo_fr *shifts = (lo_fr *)malloc(sizeof(lo_fr) * (w > q ? w : q));
    for (size_t c = 0; c < w; ++c) shifts[c] = GEN;
    lo_fr *lde = (lo_fr *)malloc(sizeof(lo_fr) * N * w);
    lo_coset_lde_batch(trace, h, w, lb, shifts, lde, nthreads);
    lo_phase("trace LDE", &tph);
    lo_fr *tlay = (lo_fr *)malloc(sizeof(lo_fr) * (2 * N - 1));
    lo_merkle_commit(p, lde, N, w, tlay, nthreads);
    lo_fr troot = tlay[2 * N - 2];
    lo_phase("trace tree", &tph);

    chal_t *ch = (chal_t *)malloc(sizeof(chal_t));
    ch_init(ch, p, fri->transcript);
    lo_fr x = fu(log_h);
    if (!(fri->transcript & LO_T_SKIP_LOG_DEGREE)) ch_observe(ch, &x);
    ch_observe(ch, &troot);
    if (!(fri->transcript & LO_T_SKIP_PUBLIC)) {
        ch_observe(ch, &p->alpha);
        ch_observe(ch, &p->delta);
    }
    lo_fr alpha = ch_sample(ch);

    /* ---- quotient */
    size_t per = q; /* Z_H takes q distinct values on the coset */
    lo_fr *zh = (lo_fr *)malloc(sizeof(lo_fr) * per), *invz = (lo_fr *)malloc(sizeof(lo_fr) * per);
    {
        lo_fr spow, gr = two_adic_gen(log_q), g = ONE;
        fpow64(&GEN, h, &spow);
        for (size_t k = 0; k < per; ++k) {
            fmul(&spow, &g, &zh[k]);
            fsub(&zh[k], &ONE, &zh[k]);
            fmul(&g, &gr, &g);
        }
        batch_inverse(zh, invz, per, 1);
    }
    lo_fr *xsq = (lo_fr *)malloc(sizeof(lo_fr) * Q), *first = (lo_fr *)malloc(sizeof(lo_fr) * Q),
          *last = (lo_fr *)malloc(sizeof(lo_fr) * Q), *trans = (lo_fr *)malloc(sizeof(lo_fr) * Q),
          *tmp = (lo_fr *)malloc(sizeof(lo_fr) * Q);
    powers(two_adic_gen(logQ), Q, xsq, nthreads);
    lo_fr wh = two_adic_gen(log_h), whinv;
    finv(&wh, &whinv);
    for (size_t i = 0; i < Q; ++i) fmul(&xsq[i], &GEN, &xsq[i]);
    for (size_t i = 0; i < Q; ++i) fsub(&xsq[i], &ONE, &tmp[i]);
    batch_inverse(tmp, first, Q, nthreads);
    for (size_t i = 0; i < Q; ++i) fsub(&xsq[i], &whinv, &trans[i]);
    batch_inverse(trans, last, Q, nthreads);
    for (size_t i = 0; i < Q; ++i) {
        fmul(&first[i], &zh[i % per], &first[i]);
        fmul(&last[i], &zh[i % per], &last[i]);
    }
    lo_phase("quotient selectors", &tph);
    lo_fr *qv = (lo_fr *)malloc(sizeof(lo_fr) * Q);
    q_ctx qc = {cfgs, ncfg, lde, w, logQ, log_q, first, last, trans, invz, &p->alpha, &p->delta, &alpha, qv, Q};
    parallel_for(Q, nthreads, q_range, &qc);
    free(xsq); free(first); free(last); free(trans); free(tmp); free(zh); free(invz);
    lo_phase("quotient values", &tph);

    /* ---- commit to quotient chunks: qv viewed as h x q row-major */
    lo_fr gq = two_adic_gen(logQ), gqinv;
    finv(&gq, &gqinv);
    shifts[0] = ONE;
    for (size_t j = 1; j < q; ++j) fmul(&shifts[j - 1], &gqinv, &shifts[j]);
    lo_fr *qlde = (lo_fr *)malloc(sizeof(lo_fr) * N * q);
    lo_coset_lde_batch(qv, h, q, lb, shifts, qlde, nthreads);
    lo_phase("quotient LDE", &tph);
    lo_fr *qlay = (lo_fr *)malloc(sizeof(lo_fr) * (2 * N - 1));
    lo_merkle_commit(p, qlde, N, q, qlay, nthreads);
    lo_fr qroot = qlay[2 * N - 2];
    lo_phase("quotient tree", &tph);
    ch_observe(ch, &qroot);
    lo_fr zeta = ch_sample(ch), zeta_next;
    fmul(&zeta, &wh, &zeta_next);

    /* ---- open (alpha_fri is sampled after the opened values: U7) */
    lo_fr *xs = (lo_fr *)malloc(sizeof(lo_fr) * N), *xs_nat = (lo_fr *)malloc(sizeof(lo_fr) * N);
    powers(two_adic_gen(logN), N, xs_nat, nthreads);
    xs_ctx xc = {xs_nat, xs, logN};
    parallel_for(N, nthreads, xs_range, &xc);
    free(xs_nat);
    lo_fr *den = (lo_fr *)malloc(sizeof(lo_fr) * N), *invd_z = (lo_fr *)malloc(sizeof(lo_fr) * N),
          *invd_zn = (lo_fr *)malloc(sizeof(lo_fr) * N);
    den_ctx dc = {xs, zeta, den};
    parallel_for(N, nthreads, den_range, &dc);
    batch_inverse(den, invd_z, N, nthreads);
    dc.z = zeta_next;
    parallel_for(N, nthreads, den_range, &dc);
    batch_inverse(den, invd_zn, N, nthreads);
    free(den);
    lo_phase("open: points, inverses", &tph);

    lo_fr *ys_z = (lo_fr *)malloc(sizeof(lo_fr) * w), *ys_zn = (lo_fr *)malloc(sizeof(lo_fr) * w),
          *ys_q = (lo_fr *)malloc(sizeof(lo_fr) * q);
    interpolate(lde, h, w, xs, invd_z, &zeta, ys_z);
    interpolate(lde, h, w, xs, invd_zn, &zeta_next, ys_zn);
    interpolate(qlde, h, q, xs, invd_z, &zeta, ys_q);
    if (fri->transcript & LO_T_OBSERVE_OPENED) {
        for (size_t c = 0; c < w; ++c) ch_observe(ch, &ys_z[c]);
        for (size_t c = 0; c < w; ++c) ch_observe(ch, &ys_zn[c]);
        for (size_t j = 0; j < q; ++j) ch_observe(ch, &ys_q[j]);
    }
    lo_fr alpha_fri = ch_sample(ch);
    lo_phase("open: opened values", &tph);

    size_t nap = 2 * w + q + 1;
    lo_fr *apw = (lo_fr *)malloc(sizeof(lo_fr) * nap);
    apw[0] = ONE;
    for (size_t k = 1; k < nap; ++k) fmul(&apw[k - 1], &alpha_fri, &apw[k]);
    red_ctx rc;
    rc.lde = lde; rc.qlde = qlde; rc.w = w; rc.q = q; rc.invz = invd_z; rc.invzn = invd_zn; rc.apw = apw;
    rc.ry_z = ZERO_FR; rc.ry_zn = ZERO_FR;
    for (size_t k = 0; k < w; ++k) {
        lo_fr t;
        fmul(&apw[k], &ys_z[k], &t);
        fadd(&rc.ry_z, &t, &rc.ry_z);
        fmul(&apw[k], &ys_zn[k], &t);
        fadd(&rc.ry_zn, &t, &rc.ry_zn);
    }
    rc.ryq = ys_q; /* width-1 matrices: reduced_ys = y */
    lo_fr *ro = (lo_fr *)malloc(sizeof(lo_fr) * N);
    rc.ro = ro;
    parallel_for(N, nthreads, red_range, &rc);
    if (dbg && dbg->fri_input) memcpy(dbg->fri_input, ro, sizeof(lo_fr) * N);
    free(invd_z); free(invd_zn); free(xs);
    lo_phase("open: reduce rows", &tph);

    /* ---- FRI commit phase */
    size_t final_len = (size_t)1 << (lb + fri->log_final_poly_len);
    uint32_t nrounds = 0;
    for (size_t len = N; len > final_len; len >>= 1) nrounds++;
    lo_fr **flay = (lo_fr **)calloc(nrounds + 1, sizeof(lo_fr *));
    lo_fr *froots = (lo_fr *)malloc(sizeof(lo_fr) * (nrounds + 1));
    lo_fr *cur = ro, *nxtv = NULL;
    lo_fr half = fu(2);
    finv(&half, &half);
    size_t len = N;
    for (uint32_t r = 0; r < nrounds; ++r) {
        size_t m = len / 2;
        flay[r] = (lo_fr *)malloc(sizeof(lo_fr) * (2 * m - 1));
        lo_merkle_commit(p, cur, m, 2, flay[r], nthreads);
        froots[r] = flay[r][2 * m - 2];
        ch_observe(ch, &froots[r]);
        lo_fr beta = ch_sample(ch);
        /* fold */
        lo_fr g = two_adic_gen(log2_strict(m) + 1), ginv;
        finv(&g, &ginv);
        lo_fr *gp = (lo_fr *)malloc(sizeof(lo_fr) * m);
        powers(ginv, m, gp, nthreads);
        nxtv = (lo_fr *)malloc(sizeof(lo_fr) * m);
        fold_ctx fc;
        fc.v = cur; fc.o = nxtv; fc.half = half; fc.gpow = gp; fc.logm = log2_strict(m);
        fmul(&beta, &half, &fc.hb);
        parallel_for(m, nthreads, fold_range, &fc);
        free(gp);
        /* keep the round's vector (leaves) for query openings */
        flay[nrounds] = NULL;
        if (r > 0) { /* cur is owned by us after round 0 (round 0 input is ro) */ }
        /* stash: we need the leaf values of each round: store them after the layers */
        lo_fr *keep = (lo_fr *)realloc(flay[r], sizeof(lo_fr) * (2 * m - 1 + len));
        memcpy(keep + (2 * m - 1), cur, sizeof(lo_fr) * len);
        flay[r] = keep;
        if (cur != ro) free(cur);
        cur = nxtv;
        len = m;
    }
    /* final poly: bit-reverse, IDFT, truncate */
    size_t flen = (size_t)1 << fri->log_final_poly_len;
    lo_fr *fin = (lo_fr *)malloc(sizeof(lo_fr) * len);
    uint32_t lgl = log2_strict(len);
    for (size_t i = 0; i < len; ++i) fin[i] = cur[bitrev64(i, lgl)];
    lo_fr winv = two_adic_gen(lgl), linv = fu(len);
    finv(&winv, &winv);
    finv(&linv, &linv);
    ntt_inplace(fin, len, &winv);
    for (size_t i = 0; i < len; ++i) fmul(&fin[i], &linv, &fin[i]);
    for (size_t i = flen; i < len; ++i)
        if (!fis_zero(&fin[i])) return -4; /* final poly degree too high */
    if (!(fri->transcript & LO_T_SKIP_FINAL_POLY))
        for (size_t i = 0; i < flen; ++i) ch_observe(ch, &fin[i]);
    lo_phase("FRI commit phase", &tph);
    uint64_t pw = ch_grind(ch, fri->pow_bits);
    if (cur != ro) free(cur);

    /* ---- serialize */
    buf_t b = {NULL, 0, 0};
    bput(&b, "LSPPRF02", 8);
    bput_u32(&b, log_h);
    bput_u32(&b, log_q);
    bput_u32(&b, (uint32_t)w);
    bput_u32(&b, fri->num_queries);
    bput_u32(&b, nrounds);
    bput_u32(&b, (uint32_t)flen);
    bput_fr(&b, &troot);
    bput_fr(&b, &qroot);
    for (size_t c = 0; c < w; ++c) bput_fr(&b, &ys_z[c]);
    for (size_t c = 0; c < w; ++c) bput_fr(&b, &ys_zn[c]);
    for (size_t j = 0; j < q; ++j) bput_fr(&b, &ys_q[j]);
    for (uint32_t r = 0; r < nrounds; ++r) bput_fr(&b, &froots[r]);
    for (size_t i = 0; i < flen; ++i) bput_fr(&b, &fin[i]);
    lo_fr pwf = fu(pw);
    bput_fr(&b, &pwf);
    for (uint32_t qi = 0; qi < fri->num_queries; ++qi) {
        size_t idx = (size_t)ch_sample_bits(ch, logN);
        for (size_t c = 0; c < w; ++c) bput_fr(&b, &lde[idx * w + c]);
        tree_path(tlay, N, idx, &b);
        for (size_t j = 0; j < q; ++j) bput_fr(&b, &qlde[idx * q + j]);
        tree_path(qlay, N, idx, &b);
        size_t l2 = N;
        for (uint32_t r = 0; r < nrounds; ++r) {
            size_t m = l2 / 2, ii = idx >> r;
            const lo_fr *leafv = flay[r] + (2 * m - 1);
            bput_fr(&b, &leafv[ii ^ 1]);
            tree_path(flay[r], m, ii >> 1, &b);
            l2 = m;
        }
    }
    if (dbg) {
        if (dbg->trace_lde) memcpy(dbg->trace_lde, lde, sizeof(lo_fr) * N * w);
        if (dbg->trace_layers) memcpy(dbg->trace_layers, tlay, sizeof(lo_fr) * (2 * N - 1));
        if (dbg->quotient) memcpy(dbg->quotient, qv, sizeof(lo_fr) * Q);
        if (dbg->quotient_lde) memcpy(dbg->quotient_lde, qlde, sizeof(lo_fr) * N * q);
        if (dbg->quotient_layers) memcpy(dbg->quotient_layers, qlay, sizeof(lo_fr) * (2 * N - 1));
        dbg->challenges[0] = alpha;
        dbg->challenges[1] = zeta;
        dbg->challenges[2] = alpha_fri;
        dbg->challenges[3] = fin[0];
    }
    for (uint32_t r = 0; r < nrounds; ++r) free(flay[r]);
    free(flay); free(froots); free(fin); free(apw); free(ro); free(ys_z); free(ys_zn); free(ys_q);
    free(qlde); free(qlay); free(qv); free(lde); free(tlay); free(shifts); free(ch);
    lo_phase("grind, queries, serialize", &tph);
    *proof_out = b.b;
    *proof_len = b.n;
    return 0;
}

/* --------------------------------------------------------------- verifier */
typedef struct { const uint8_t *b; size_t n, off; int bad; } rd_t;
static uint32_t rd_u32(rd_t *r) {
    uint32_t x = 0;
    if (r->off + 4 > r->n) { r->bad = 1; return 0; }
    memcpy(&x, r->b + r->off, 4);
    r->off += 4;
    return x;
}
static lo_fr rd_fr(rd_t *r) {
    uint64_t c[4] = {0, 0, 0, 0};
    lo_fr o = ZERO_FR;
    if (r->off + 32 > r->n) { r->bad = 1; return o; }
    memcpy(c, r->b + r->off, 32);
    r->off += 32;
    if (geq_mod(c)) { r->bad = 1; return o; }
    lo_fr_from_canonical(c, &o);
    return o;
}
static int mk_verify(const lo_params *p, const lo_fr *root, size_t index, const lo_fr *leaf, size_t nleaf,
                     rd_t *r, uint32_t expect_len) {
    uint32_t pl = rd_u32(r);
    if (pl != expect_len) return 0;
    lo_fr cur;
    lo_hash_iter(p, leaf, nleaf, &cur);
    for (uint32_t i = 0; i < pl; ++i) {
        lo_fr sib = rd_fr(r);
        if ((index >> i) & 1) compress2(p, &sib, &cur, &cur);
        else compress2(p, &cur, &sib, &cur);
    }
    return !r->bad && feq(&cur, root);
}

int lo_verify(const lo_params *p, const lo_fri *fri, const int32_t *air, size_t air_len, int public_degree,
              const uint8_t *proof, size_t proof_len) {
    field_init();
    GEN = fu(22);
    static cfg_t cfgs[MAXCFG];
    int ncfg, K;
    if (parse_air(air, air_len, cfgs, &ncfg)) return -1;
    rd_t r = {proof, proof_len, 0, 0};
    if (proof_len < 8 || memcmp(proof, "LSPPRF02", 8)) return 1;
    r.off = 8;
    uint32_t log_h = rd_u32(&r), log_q = rd_u32(&r), w = rd_u32(&r), nq = rd_u32(&r), nr = rd_u32(&r),
             nf = rd_u32(&r);
    if (nf != 1) return 3; /* this verifier reads a 1-coefficient final polynomial only */
    int maxd = constraint_stats(cfgs, ncfg, public_degree, &K);
    if (maxd < 2) maxd = 2;
    uint32_t elq = 0;
    while ((1 << elq) < maxd - 1) ++elq;
    if (r.bad || elq != log_q || nq != fri->num_queries || log_h > 40 || w > 4096) return 2;
    uint32_t lb = fri->log_blowup, logN = log_h + lb;
    if (nr != logN - lb - fri->log_final_poly_len) return 3;
    size_t q = (size_t)1 << log_q, h = (size_t)1 << log_h;
    lo_fr troot = rd_fr(&r), qroot = rd_fr(&r);
    lo_fr *tl = (lo_fr *)malloc(sizeof(lo_fr) * w), *tn = (lo_fr *)malloc(sizeof(lo_fr) * w),
          *qc = (lo_fr *)malloc(sizeof(lo_fr) * q), *roots = (lo_fr *)malloc(sizeof(lo_fr) * (nr + 1)),
          *betas = (lo_fr *)malloc(sizeof(lo_fr) * (nr + 1));
    for (uint32_t c = 0; c < w; ++c) tl[c] = rd_fr(&r);
    for (uint32_t c = 0; c < w; ++c) tn[c] = rd_fr(&r);
    for (size_t j = 0; j < q; ++j) qc[j] = rd_fr(&r);
    for (uint32_t k = 0; k < nr; ++k) roots[k] = rd_fr(&r);
    lo_fr fp = rd_fr(&r), pwf = rd_fr(&r);
    int rc = 0;
    chal_t *ch = (chal_t *)malloc(sizeof(chal_t));
    ch_init(ch, p, fri->transcript);
    lo_fr x = fu(log_h);
    if (!(fri->transcript & LO_T_SKIP_LOG_DEGREE)) ch_observe(ch, &x);
    ch_observe(ch, &troot);
    if (!(fri->transcript & LO_T_SKIP_PUBLIC)) {
        ch_observe(ch, &p->alpha);
        ch_observe(ch, &p->delta);
    }
    lo_fr alpha = ch_sample(ch);
    ch_observe(ch, &qroot);
    lo_fr zeta = ch_sample(ch), wh = two_adic_gen(log_h), zeta_next, whinv;
    fmul(&zeta, &wh, &zeta_next);
    finv(&wh, &whinv);
    if (fri->transcript & LO_T_OBSERVE_OPENED) {
        for (uint32_t c = 0; c < w; ++c) ch_observe(ch, &tl[c]);
        for (uint32_t c = 0; c < w; ++c) ch_observe(ch, &tn[c]);
        for (size_t j = 0; j < q; ++j) ch_observe(ch, &qc[j]);
    }
    lo_fr alpha_fri = ch_sample(ch);
    for (uint32_t k = 0; k < nr; ++k) {
        ch_observe(ch, &roots[k]);
        betas[k] = ch_sample(ch);
    }
    if (!(fri->transcript & LO_T_SKIP_FINAL_POLY)) ch_observe(ch, &fp);
    uint64_t pwc[4];
    lo_fr_to_canonical(&pwf, pwc);
    if (pwc[1] | pwc[2] | pwc[3]) { rc = 4; goto done; }
    if (!ch_check_witness(ch, fri->pow_bits, pwc[0])) { rc = 5; goto done; }
    {
        lo_fr gN = two_adic_gen(logN);
        lo_fr *trow = (lo_fr *)malloc(sizeof(lo_fr) * w), *qrow = (lo_fr *)malloc(sizeof(lo_fr) * q);
        for (uint32_t qi = 0; qi < nq && !rc; ++qi) {
            size_t idx = (size_t)ch_sample_bits(ch, logN);
            for (uint32_t c = 0; c < w; ++c) trow[c] = rd_fr(&r);
            if (!mk_verify(p, &troot, idx, trow, w, &r, logN)) { rc = 6; break; }
            for (size_t j = 0; j < q; ++j) qrow[j] = rd_fr(&r);
            if (!mk_verify(p, &qroot, idx, qrow, q, &r, logN)) { rc = 7; break; }
            lo_fr xq, t, u, ro = ZERO_FR, apow = ONE, dz, dzn;
            fpow64(&gN, bitrev64(idx, logN), &xq);
            fmul(&xq, &GEN, &xq);
            fsub(&xq, &zeta, &dz);
            finv(&dz, &dz);
            fsub(&xq, &zeta_next, &dzn);
            finv(&dzn, &dzn);
            for (uint32_t c = 0; c < w; ++c) {
                fsub(&trow[c], &tl[c], &t);
                fmul(&t, &dz, &t);
                fmul(&t, &apow, &t);
                fadd(&ro, &t, &ro);
                fmul(&apow, &alpha_fri, &apow);
            }
            for (uint32_t c = 0; c < w; ++c) {
                fsub(&trow[c], &tn[c], &t);
                fmul(&t, &dzn, &t);
                fmul(&t, &apow, &t);
                fadd(&ro, &t, &ro);
                fmul(&apow, &alpha_fri, &apow);
            }
            for (size_t j = 0; j < q; ++j) {
                fsub(&qrow[j], &qc[j], &t);
                fmul(&t, &dz, &t);
                fmul(&t, &apow, &t);
                fadd(&ro, &t, &ro);
                fmul(&apow, &alpha_fri, &apow);
            }
            lo_fr folded = ro;
            size_t index = idx;
            for (uint32_t k = 0; k < nr; ++k) {
                uint32_t log_folded = logN - 1 - k;
                lo_fr ev[2];
                lo_fr sib = rd_fr(&r);
                ev[(index ^ 1) & 1] = sib;
                ev[index & 1] = folded;
                if (!mk_verify(p, &roots[k], index >> 1, ev, 2, &r, log_folded)) { rc = 8; break; }
                index >>= 1;
                /* fold_row */
                lo_fr g2 = two_adic_gen(log_folded + 1), s0, s1, num, den;
                fpow64(&g2, bitrev64(index, log_folded), &s0);
                fsub(&ZERO_FR, &s0, &s1);
                fsub(&betas[k], &s0, &u);
                fsub(&ev[1], &ev[0], &num);
                fmul(&u, &num, &u);
                fsub(&s1, &s0, &den);
                finv(&den, &den);
                fmul(&u, &den, &u);
                fadd(&ev[0], &u, &folded);
            }
            if (rc) break;
            if (!feq(&folded, &fp)) { rc = 9; break; }
        }
        free(trow);
        free(qrow);
        if (rc) goto done;
    }
    if (r.bad || r.off != r.n) { rc = 10; goto done; }
    {
        /* out-of-domain quotient identity */
        lo_fr gq = two_adic_gen(log_h + log_q), quotient = ZERO_FR, t, u;
        lo_fr *sh = (lo_fr *)malloc(sizeof(lo_fr) * q);
        sh[0] = GEN;
        for (size_t j = 1; j < q; ++j) fmul(&sh[j - 1], &gq, &sh[j]);
        for (size_t i = 0; i < q; ++i) {
            lo_fr prod = ONE;
            for (size_t j = 0; j < q; ++j) {
                if (j == i) continue;
                lo_fr si, a, b2;
                finv(&sh[j], &si);
                fmul(&zeta, &si, &a);
                fpow64(&a, h, &a);
                fsub(&a, &ONE, &a);
                fmul(&sh[i], &si, &b2);
                fpow64(&b2, h, &b2);
                fsub(&b2, &ONE, &b2);
                finv(&b2, &b2);
                fmul(&prod, &a, &prod);
                fmul(&prod, &b2, &prod);
            }
            fmul(&prod, &qc[i], &t);
            fadd(&quotient, &t, &quotient);
        }
        free(sh);
        lo_fr zh, first, last, trans, acc = ZERO_FR;
        fpow64(&zeta, h, &zh);
        fsub(&zh, &ONE, &zh);
        fsub(&zeta, &ONE, &t);
        finv(&t, &t);
        fmul(&zh, &t, &first);
        fsub(&zeta, &whinv, &trans);
        finv(&trans, &t);
        fmul(&zh, &t, &last);
        eval_fold(cfgs, ncfg, tl, tn, &p->alpha, &p->delta, &first, &last, &trans, &alpha, &acc);
        finv(&zh, &u);
        fmul(&acc, &u, &acc);
        if (!feq(&acc, &quotient)) rc = 11;
    }
done:
    free(tl); free(tn); free(qc); free(roots); free(betas); free(ch);
    return rc;
}

/* ------------------------------------------------------- synthetic trace */
int lo_gen_perm_trace(uint32_t log_n, uint32_t ncols, const lo_fr *alpha, const lo_fr *delta,
                      uint64_t seed, int small, lo_fr *rows) {
    field_init();
    size_t n = (size_t)1 << log_n, w = 2 * ncols + 2;
    smix r = {seed ^ 0x5452414345ULL};
    lo_fr *a = (lo_fr *)malloc(sizeof(lo_fr) * n * ncols);
    for (uint32_t c = 0; c < ncols; ++c)
        for (size_t i = 0; i < n; ++i) a[c * n + i] = small ? fu(smix_next(&r) & 0xFFFFFFFFULL) : smix_fr(&r);
    size_t *perm = (size_t *)malloc(sizeof(size_t) * n);
    for (size_t i = 0; i < n; ++i) perm[i] = i;
    for (size_t i = n - 1; i > 0; --i) {
        size_t j = (size_t)smix_below(&r, i + 1);
        size_t t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
    lo_fr prev = ONE;
    lo_fr *den = (lo_fr *)malloc(sizeof(lo_fr) * n), *binv = (lo_fr *)malloc(sizeof(lo_fr) * n);
    for (size_t i = 0; i < n; ++i) {
        lo_fr *row = rows + i * w;
        lo_fr bc = ZERO_FR;
        for (uint32_t c = 0; c < ncols; ++c) {
            row[c] = a[c * n + i];
            row[ncols + c] = a[c * n + perm[i]];
            fmul(&bc, alpha, &bc);
            fadd(&bc, &row[ncols + c], &bc);
        }
        fadd(&bc, delta, &den[i]);
    }
    batch_inverse(den, binv, n, 8);
    for (size_t i = 0; i < n; ++i) {
        lo_fr *row = rows + i * w;
        lo_fr ac = ZERO_FR;
        for (uint32_t c = 0; c < ncols; ++c) {
            fmul(&ac, alpha, &ac);
            fadd(&ac, &row[c], &ac);
        }
        fadd(&ac, delta, &ac);
        row[2 * ncols] = binv[i];
        fmul(&prev, &ac, &prev);
        fmul(&prev, &binv[i], &prev);
        row[2 * ncols + 1] = prev;
    }
    int ok = feq(&prev, &ONE);
    free(a); free(perm); free(den); free(binv);
    return ok ? 0 : -1;
}
