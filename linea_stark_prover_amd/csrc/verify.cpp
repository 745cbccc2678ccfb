// Host CPU verifier: p3_uni_stark::verify (bin/src/main.rs:88-96) with
// TwoAdicFriPcs::verify and the FRI query checks ([EXT p3-fri]).  The
// reference verifies in ~1 s on the CPU (bench.log:69); it stays on the host.
#include <cstring>

#include "prove_internal.hpp"

namespace lsp {

namespace {
struct Reader {
    const uint8_t* b;
    size_t n, off = 0;
    bool bad = false;
    uint32_t u32() {
        if (off + 4 > n) {
            bad = true;
            return 0;
        }
        uint32_t x = 0;
        for (int i = 0; i < 4; ++i) x |= (uint32_t)b[off + i] << (8 * i);
        off += 4;
        return x;
    }
    Fr fr() {
        Fr c = fr_zero();
        if (off + 32 > n) {
            bad = true;
            return c;
        }
        for (int i = 0; i < 8; ++i) {
            uint32_t x = 0;
            for (int k = 0; k < 4; ++k) x |= (uint32_t)b[off + 4 * i + k] << (8 * k);
            c.v[i] = x;
        }
        off += 32;
        if (!fr_words_lt_mod(c)) {
            bad = true;
            return fr_zero();
        }
        return fr_from_canonical(c);
    }
};

bool mk_verify(const P2Host& p2, const Fr& root, size_t index, const Fr* leaf, size_t nleaf, Reader& r,
               uint32_t expect) {
    const uint32_t pl = r.u32();
    if (pl != expect) return false;
    Fr cur = p2.hash(leaf, nleaf);
    for (uint32_t i = 0; i < pl; ++i) {
        const Fr sib = r.fr();
        cur = ((index >> i) & 1) ? p2.compress(sib, cur) : p2.compress(cur, sib);
    }
    return !r.bad && fr_eq(cur, root);
}
}  // namespace

int verify_host(const lsp_ctx* ctx, const Air& air, const Fr* pub, size_t npub, const uint8_t* b, size_t n) {
    if (npub < 2) return 1;
    if (n < 8 || std::memcmp(b, "LSPPRF02", 8) != 0) return 2;
    Reader r{b, n};
    r.off = 8;
    const uint32_t log_h = r.u32(), log_q = r.u32(), w = r.u32(), nq = r.u32(), nr = r.u32(), nf = r.u32();
    if (r.bad || log_q != air.log_quotient_degree(ctx->public_degree) || nq != ctx->num_queries || log_h > 40 ||
        log_h < 1 || w <= air.max_col || w > (1u << 20))
        return 3;
    const uint32_t lb = ctx->log_blowup, logN = log_h + lb;
    if (nr != logN - lb - ctx->log_final_poly_len || nf != (1u << ctx->log_final_poly_len)) return 4;
    const size_t q = (size_t)1 << log_q, h = (size_t)1 << log_h;
    const size_t flen = (size_t)1 << ctx->log_final_poly_len;
    const Fr troot = r.fr(), qroot = r.fr();
    std::vector<Fr> tl(w), tn(w), qc(q), roots(nr), betas(nr), fp(flen);
    for (auto& x : tl) x = r.fr();
    for (auto& x : tn) x = r.fr();
    for (auto& x : qc) x = r.fr();
    for (auto& x : roots) x = r.fr();
    for (auto& x : fp) x = r.fr();
    const Fr pw = r.fr();
    if (r.bad) return 5;
    const Fr one = fr_one(), GEN = host_generator();
    const TranscriptCfg& TC = ctx->transcript;  // U7 / U8 / U12, as the prover
    Challenger ch(&ctx->p2, TC.mont_bits);
    if (TC.log_degree) ch.observe(fr_from_u64(log_h));
    ch.observe(troot);
    if (TC.public_values)
        for (size_t i = 0; i < npub; ++i) ch.observe(pub[i]);
    const Fr alpha = ch.sample();
    ch.observe(qroot);
    const Fr zeta = ch.sample();
    const Fr wh = host_two_adic_generator(log_h), wh_inv = fr_inv(wh);
    const Fr zeta_next = fr_mul(zeta, wh);
    if (TC.opened_values) {
        for (const Fr& v : tl) ch.observe(v);
        for (const Fr& v : tn) ch.observe(v);
        for (const Fr& v : qc) ch.observe(v);
    }
    const Fr alpha_fri = ch.sample();
    for (uint32_t k = 0; k < nr; ++k) {
        ch.observe(roots[k]);
        betas[k] = ch.sample();
    }
    if (TC.final_poly)
        for (auto& c : fp) ch.observe(c);
    const Fr pwc = fr_to_canonical(pw);
    for (int i = 2; i < 8; ++i)
        if (pwc.v[i]) return 6;
    if (!ch.check_witness(ctx->pow_bits, (uint64_t)pwc.v[0] | ((uint64_t)pwc.v[1] << 32))) return 7;
    const Fr gN = host_two_adic_generator(logN);
    std::vector<Fr> trow(w), qrow(q);
    for (uint32_t qi = 0; qi < nq; ++qi) {
        const size_t idx = (size_t)ch.sample_bits(logN);
        for (auto& x : trow) x = r.fr();
        if (!mk_verify(ctx->p2, troot, idx, trow.data(), w, r, logN)) return 8;
        for (auto& x : qrow) x = r.fr();
        if (!mk_verify(ctx->p2, qroot, idx, qrow.data(), q, r, logN)) return 9;
        const Fr x = fr_mul(GEN, fr_pow_u64(gN, host_bitrev(idx, logN)));
        const Fr dz = fr_inv(fr_sub(x, zeta)), dzn = fr_inv(fr_sub(x, zeta_next));
        Fr ro = fr_zero(), apow = one;
        for (uint32_t c = 0; c < w; ++c) {
            ro = fr_add(ro, fr_mul(apow, fr_mul(fr_sub(trow[c], tl[c]), dz)));
            apow = fr_mul(apow, alpha_fri);
        }
        for (uint32_t c = 0; c < w; ++c) {
            ro = fr_add(ro, fr_mul(apow, fr_mul(fr_sub(trow[c], tn[c]), dzn)));
            apow = fr_mul(apow, alpha_fri);
        }
        for (size_t j = 0; j < q; ++j) {
            ro = fr_add(ro, fr_mul(apow, fr_mul(fr_sub(qrow[j], qc[j]), dz)));
            apow = fr_mul(apow, alpha_fri);
        }
        Fr folded = ro;
        size_t index = idx;
        for (uint32_t k = 0; k < nr; ++k) {
            const uint32_t log_folded = logN - 1 - k;
            Fr ev[2];
            ev[(index ^ 1) & 1] = r.fr();
            ev[index & 1] = folded;
            if (!mk_verify(ctx->p2, roots[k], index >> 1, ev, 2, r, log_folded)) return 10;
            index >>= 1;
            // TwoAdicFriGenericConfig::fold_row
            const Fr s0 = fr_pow_u64(host_two_adic_generator(log_folded + 1), host_bitrev(index, log_folded));
            const Fr s1 = fr_neg(s0);
            folded = fr_add(ev[0], fr_mul(fr_mul(fr_sub(betas[k], s0), fr_sub(ev[1], ev[0])),
                                          fr_inv(fr_sub(s1, s0))));
        }
        // final polynomial at x^(2^nr) (constant when log_final_poly_len = 0)
        const Fr xf = fr_pow_u64(host_two_adic_generator(logN - nr), host_bitrev(index, logN - nr));
        Fr ev = fr_zero();
        for (size_t k = flen; k-- > 0;) ev = fr_add(fr_mul(ev, xf), fp[k]);
        if (!fr_eq(ev, folded)) return 11;
    }
    if (r.bad || r.off != r.n) return 12;
    // out-of-domain identity: folded_constraints(zeta) / Z_H(zeta) == sum zps_i * chunk_i
    const Fr gQ = host_two_adic_generator(log_h + log_q);
    std::vector<Fr> sh(q);
    sh[0] = GEN;
    for (size_t j = 1; j < q; ++j) sh[j] = fr_mul(sh[j - 1], gQ);
    auto zp = [&](const Fr& s, const Fr& xx) { return fr_sub(fr_pow_u64(fr_mul(xx, fr_inv(s)), h), one); };
    Fr quotient = fr_zero();
    for (size_t i = 0; i < q; ++i) {
        Fr prod = one;
        for (size_t j = 0; j < q; ++j)
            if (j != i) prod = fr_mul(prod, fr_mul(zp(sh[j], zeta), fr_inv(zp(sh[j], sh[i]))));
        quotient = fr_add(quotient, fr_mul(prod, qc[i]));
    }
    const Fr zh = fr_sub(fr_pow_u64(zeta, h), one);
    const Fr first = fr_mul(zh, fr_inv(fr_sub(zeta, one)));
    const Fr last = fr_mul(zh, fr_inv(fr_sub(zeta, wh_inv)));
    const Fr trans = fr_sub(zeta, wh_inv);
    Fr acc = fr_zero();
    air.eval_fold(tl.data(), tn.data(), pub[0], pub[1], first, last, trans, alpha, acc);
    if (!fr_eq(fr_mul(acc, fr_inv(zh)), quotient)) return 13;
    return 0;
}

}  // namespace lsp
