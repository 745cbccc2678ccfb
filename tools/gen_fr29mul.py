"""Generate linea_stark_prover_amd/csrc/fr29_mul_gfx950.inc: the 29-bit-limb
Montgomery product and square (fr29.hpp) with each FIPS column as one inline
asm block of chained v_mad_u64_u32 on one 64-bit accumulator (CHAINS = 1) or
two (CHAINS = 2, summed at the column end).

Left to itself the compiler splits every column into several partial
accumulators and recombines them with v_lshl_add_u64 (~29 extra VALU ops per
product); the asm keeps the column on the accumulator chain.  The quotient
digits m_k are full 32-bit words (-acc mod 2^32, no mask): column sums stay
below 2^63.2 (9 products of normalised limbs, 8 products m_j r_i < 2^32 r_i,
m_k and the carry -- tools/gen_fr29mul.py --bound), so the MAD carry-out is
never needed (it goes to a scratch SGPR pair).

Run:  python tools/gen_fr29mul.py [chains]   (rewrites the .inc; commit it)
"""
import math
import os
import sys

P29 = [0x1, 0x108c0000, 0x42, 0x14edfda0, 0x1b00159a, 0x68f2e1b, 0x155982d1, 0xbd34594, 0x12ab65]
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "linea_stark_prover_amd", "csrc",
                   "fr29_mul_gfx950.inc")


def column_block(terms, chains):
    """terms: list of (x, y) operand names; returns asm lines + operand list"""
    lines, ops = [], {}
    for idx, (x, y) in enumerate(terms):
        acc = "acc" if chains == 1 or idx % 2 == 0 else "acc1"
        lines.append(f'"v_mad_u64_u32 %[{acc}], %[c], %[{x}], %[{y}], %[{acc}]\\n\\t"')
        for o in (x, y):
            ops[o] = True
    return lines, list(ops)


def operand(o):
    if o.startswith("p"):
        return f'[{o}] "s"({hex(P29[int(o[1:])])}u)'
    if o.startswith("a") or o.startswith("b"):
        return f'[{o}] "v"({o[0]}.l[{o[1:]}])'
    if o.startswith("d"):
        return f'[{o}] "v"(d{o[1:]})'
    return f'[{o}] "v"({o})'  # m_j


def gen(kind, chains):
    sq = kind == "sqr"
    name = "f29_sqr_asm" if sq else "f29_mul_asm"
    sig = "(const F29& a)" if sq else "(const F29& a, const F29& b)"
    out = [f"__device__ __forceinline__ F29 {name}{sig} {{"]
    out.append("    uint32_t m0, m1, m2, m3, m4, m5, m6, m7, m8;")
    if sq:
        out.append("    const uint32_t " + ", ".join(f"d{i} = a.l[{i}] << 1" for i in range(9)) + ";")
    out.append("    F29 o;")
    out.append("    uint64_t acc = 0, c;")
    if chains == 2:
        out.append("    uint64_t acc1;")
    for k in range(17):
        terms = []
        if sq:
            for i in range(max(0, k - 8), 9):
                j = k - i
                if j < 0 or j > 8 or i >= j:
                    continue
                terms.append((f"d{i}", f"a{j}"))
            if k % 2 == 0 and k // 2 <= 8:
                terms.append((f"a{k // 2}", f"a{k // 2}"))
        else:
            for j in range(max(0, k - 8), min(k, 8) + 1):
                terms.append((f"a{j}", f"b{k - j}"))
        for j in range(max(0, k - 8), min(k, 9)):
            if 1 <= k - j <= 8:
                terms.append((f"m{j}", f"p{k - j}"))
        if chains == 2:
            out.append("    acc1 = 0;")
        lines, ops = column_block(terms, chains)
        outs = '[acc] "+&v"(acc), [c] "=&s"(c)' + (', [acc1] "+&v"(acc1)' if chains == 2 else "")
        out.append("    asm(")
        for l in lines:
            out.append("        " + l)
        out.append(f"        : {outs}")
        out.append("        : " + ", ".join(operand(o) for o in ops) + ");")
        if chains == 2:
            out.append("    acc += acc1;")
        if k < 9:
            # 32-bit quotient digit m_k = -acc mod 2^32 (r = 1 mod 2^29, so r[0] = 1):
            # acc + m_k clears the low 32 bits, in particular the low 29
            out.append(f"    m{k} = 0u - (uint32_t)acc;")
            out.append(f'    asm("v_mad_u64_u32 %[acc], %[c], %[m], 1, %[acc]" : [acc] "+&v"(acc), [c] "=&s"(c) : [m] "v"(m{k}));')
            out.append("    acc >>= 29;")
        else:
            out.append(f"    o.l[{k - 9}] = (uint32_t)acc & F29_MASK;")
            out.append("    acc >>= 29;")
    out.append("    o.l[8] = (uint32_t)acc;")
    out.append("    (void)c;")
    out.append("    return o;")
    out.append("}")
    return out


ACC = "v[2:3]"   # block mode: the accumulator lives in a fixed, clobbered VGPR pair
ACC_LO = "v2"
ACC_HI = "v3"
R_MOD = sum(p << (29 * i) for i, p in enumerate(P29))
# the folded-digit form (--block): C = (2^261 - 1) mod r, added into the
# columns as constants (fr29.hpp, f29_mul_c)
C_OFF = ((1 << 261) - 1) % R_MOD
C29 = [(C_OFF >> (29 * i)) & ((1 << 29) - 1) for i in range(8)] + [C_OFF >> 232]


def gen_block(kind):
    """the whole product as ONE asm statement: the compiler inserts its
    conservative hazard s_nop after every asm statement whose result the next
    instruction reads; inside one statement there are none.

    Folded quotient digits (no MAD by r[0] = 1, no 64-bit shift): in a low
    column the digit is m'_k = ~acc mod 2^32, so acc + m'_k = (acc_hi + 1) 2^32
    - 1 and its floor by 2^29 is acc_hi * 8 + 7: one v_mad_u64_u32 of the high
    word by 8 that also adds the next column's constant c_(k+1) + 7.  Each low
    column of T = a b + C + M' r then ends in 29 one-bits, so the upper columns
    give Q = (T + 1) / 2^261 - 1 == a b 2^-261 (mod r) for C = (2^261 - 1) mod r
    (fr29.hpp f29_mul_c states the same in C)."""
    sq = kind == "sqr"
    name = "f29_sqr_asm" if sq else "f29_mul_asm"
    sig = "(const F29& a)" if sq else "(const F29& a, const F29& b)"
    out = [f"__device__ __forceinline__ F29 {name}{sig} {{"]
    out.append("    uint32_t m0, m1, m2, m3, m4, m5, m6, m7, m8;")
    if sq:
        # 2 a_i as v_add_u32 (2-cycle issue; the compiler's x << 1 is a 4-cycle v_lshlrev_b32)
        out.append("    uint32_t " + ", ".join(f"d{i}" for i in range(9)) + ";")
        for i in range(9):
            out.append(f'    asm("v_add_u32 %0, %1, %1" : "=v"(d{i}) : "v"(a.l[{i}]));')
    out.append("    F29 o;")
    out.append("    uint64_t c;")
    lines, ins = [], {}
    first = True
    for k in range(17):
        terms = []
        if sq:
            for i in range(max(0, k - 8), 9):
                j = k - i
                if j < 0 or j > 8 or i >= j:
                    continue
                terms.append((f"d{i}", f"a{j}"))
            if k % 2 == 0 and k // 2 <= 8:
                terms.append((f"a{k // 2}", f"a{k // 2}"))
        else:
            for j in range(max(0, k - 8), min(k, 8) + 1):
                terms.append((f"a{j}", f"b{k - j}"))
        for j in range(max(0, k - 8), min(k, 9)):
            if 1 <= k - j <= 8:
                terms.append((f"m{j}", f"p{k - j}"))
        for x, y in terms:
            src2 = "%[k0]" if first else ACC
            first = False
            lines.append(f"v_mad_u64_u32 {ACC}, %[c], %[{x}], %[{y}], {src2}")
            for o in (x, y):
                if not o.startswith("m"):
                    ins[o] = True
        if k < 9:
            lines.append(f"v_not_b32 %[m{k}], {ACC_LO}")
            lines.append(f"v_mad_u64_u32 {ACC}, %[c], {ACC_HI}, 8, %[k{k + 1}]")
        else:
            lines.append(f"v_and_b32 %[o{k - 9}], %[mask], {ACC_LO}")
            lines.append(f"v_lshrrev_b64 {ACC}, 29, {ACC}")
    lines.append(f"v_mov_b32 %[o8], {ACC_LO}")
    out.append("    asm(")
    for l in lines:
        out.append(f'        "{l}\\n\\t"')
    outs = [f'[m{k}] "=&v"(m{k})' for k in range(9)] + [f'[o{k}] "=&v"(o.l[{k}])' for k in range(9)] + ['[c] "=&s"(c)']
    consts = [f'[k0] "s"({hex(C29[0])}ull)'] + \
             [f'[k{k}] "s"({hex((C29[k] if k < 9 else 0) + 7)}ull)' for k in range(1, 10)]
    out.append("        : " + ", ".join(outs))
    out.append("        : " + ", ".join([operand(o) for o in ins] + ['[mask] "s"(0x1fffffffu)'] + consts))
    out.append('        : "v2", "v3");')
    out.append("    (void)c;")
    out.append("    (void)m0; (void)m1; (void)m2; (void)m3; (void)m4; (void)m5; (void)m6; (void)m7; (void)m8;")
    out.append("    return o;")
    out.append("}")
    return out


def bound():
    """worst column sum for normalised inputs and 32-bit quotient digits"""
    a, m, worst, carry = (1 << 29) - 1, (1 << 32) - 1, 0, 0
    for k in range(17):
        tot = sum(a * a for j in range(9) if 0 <= k - j <= 8)
        tot += sum(m * P29[k - j] for j in range(9) if 1 <= k - j <= 8) + carry + (m if k < 9 else 0)
        worst, carry = max(worst, tot), tot >> 29
    return worst


def sub16_limbs():
    """16 r with every low limb in [2^29, 2^30) (fr29.hpp f29_sub16)"""
    r = sum(p << (29 * i) for i, p in enumerate(P29))
    m = (1 << 29) - 1
    c = [(16 * r >> (29 * i)) & m for i in range(8)] + [16 * r >> (29 * 8)]
    limbs = [c[0] + (1 << 29)] + [c[i] + (1 << 29) - 1 for i in range(1, 8)] + [c[8] - 1]
    assert sum(v << (29 * i) for i, v in enumerate(limbs)) == 16 * r
    return limbs


def bound_sub16():
    """worst column sum of (a + 16r - b) * w, a normalised, w canonical"""
    r = sum(p << (29 * i) for i, p in enumerate(P29))
    L = sub16_limbs()
    a = [(1 << 29) - 1 + L[i] for i in range(8)] + [(24 * r) >> 232]
    b = [(1 << 29) - 1] * 8 + [r >> 232]
    m, worst, carry = (1 << 32) - 1, 0, 0
    for k in range(17):
        tot = sum(a[j] * b[k - j] for j in range(9) if 0 <= k - j <= 8)
        tot += sum(m * P29[k - j] for j in range(9) if 1 <= k - j <= 8) + carry + (m if k < 9 else 0)
        worst, carry = max(worst, tot), tot >> 29
    return worst


def main():
    if "--bound" in sys.argv:
        w = bound()
        print("worst column sum < 2^%.3f" % math.log2(w))
        assert w < 1 << 64
        print("f29_sub16 limbs:", ", ".join(hex(v) for v in sub16_limbs()))
        w = bound_sub16()
        print("worst column sum, (a + 16r - b) * w: < 2^%.3f" % math.log2(w))
        assert w < 1 << 64
        return
    if "--block" in sys.argv:
        out = OUT.replace(".inc", "_blk.inc")
        lines = ["// GENERATED by tools/gen_fr29mul.py --block -- do not edit by hand.",
                 "// 29-bit-limb Montgomery product / square on gfx950: FIPS, the whole product one asm",
                 "// statement (accumulator in the clobbered pair v[2:3]).  Same results as f29_mul / f29_sqr."]
        lines += gen_block("mul") + [""] + gen_block("sqr")
        with open(out, "w") as f:
            f.write("\n".join(lines) + "\n")
        print("wrote", out)
        return
    chains = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    lines = ["// GENERATED by tools/gen_fr29mul.py -- do not edit by hand.",
             f"// 29-bit-limb Montgomery product / square on gfx950: FIPS, one asm block per column,",
             f"// {chains} accumulator chain(s) per column.  Same results as f29_mul / f29_sqr."]
    lines += gen("mul", chains) + [""] + gen("sqr", chains)
    with open(OUT, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("wrote", OUT)


if __name__ == "__main__":
    main()
