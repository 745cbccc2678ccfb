"""Instruction budget of one Poseidon2 permutation in the shipped gfx950 code.

    python tools/isa_budget.py [--kernel k_merkle_level] [--json out.json]

Disassembles k_hash.o's device code (the library build, linea_stark_prover_amd/
_build/k_hash.o), takes the one-state-per-lane instance of a hash kernel
(S-box x^11, default linear layers) and reads its round loops: the loop
bodies (a backward branch each) are told apart by their v_mad_u64_u32 count
(one S-box = 3 squares x 126 + 2 products x 162 = 702 MADs; a full round =
3 S-boxes).  One permutation = 8 full-round bodies + 22 partial-round bodies
(the compiler keeps two partial-round variants: both are reported, as
bounds); what the measured SQ_INSTS_VALU per permutation holds beyond that
is the sponge's absorption and the form conversions.  Instructions are
grouped by what they are for in the 29-bit-limb arithmetic
(fr29_mul_gfx950_blk.inc, poseidon2_f29.hpp), with their share of the VALU
cycles at the rates measured on the chip (profiles/r02_rates.json: 64-bit
integer ops 4 cycles per wave64 per SIMD, 32-bit VALU 2.3).
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAD = "v_mad_u64_u32"

# (group, regex on the mnemonic), first match wins
GROUPS = [
    ("mad (products)", r"^v_mad_u64_u32$"),
    ("digit not (products)", r"^v_not_b32$"),
    ("limb split: and", r"^v_and_b32$"),
    ("limb split / carry: 64-bit shift", r"^v_lshrrev_b64$|^v_lshlrev_b64$"),
    ("32-bit shifts", r"^v_lshrrev_b32$|^v_lshlrev_b32$|^v_ashrrev_i32$|^v_alignbit_b32$|^v_bfe_u32$"),
    ("limb sums (add3/add)", r"^v_add3_u32$|^v_add_u32$|^v_add_co_u32$|^v_addc_co_u32$|^v_add_nc_u32$|^v_sub_u32$|"
                             r"^v_sub_co_u32$|^v_subb_co_u32$|^v_subrev_u32$|^v_lshl_add_u32$|^v_add_lshl_u32$"),
    ("quotient estimate (mul_hi / mul_lo)", r"^v_mul_hi_u32$|^v_mul_lo_u32$|^v_mad_u32_u24$|^v_mul_u32_u24$"),
    ("cross-lane (dpp / select)", r"dpp|^v_cndmask_b32$|^v_readlane|^v_writelane"),
    ("moves", r"^v_mov_b32$|^v_mov_b64$|^v_pk_mov_b32$"),
    ("other VALU", r"^v_"),
    ("LDS", r"^ds_"),
    ("global / buffer memory", r"^global_|^buffer_|^flat_"),
    ("scalar", r"^s_"),
]


def disassemble(obj):
    tmp = tempfile.mkdtemp()
    fat = os.path.join(tmp, "fatbin.bin")
    co = os.path.join(tmp, "dev.co")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat])
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "-unbundle", "-type=o",
                           "-targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"-input={fat}", f"-output={co}"])
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True, text=True,
                          check=True).stdout


def kernel_insts(asm, name_re):
    """[(addr, mnemonic, operands)] of the first kernel whose symbol matches"""
    out, on = [], False
    for line in asm.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.*)>:$", line)
        if m:
            if on:
                break
            on = re.search(name_re, m.group(2)) is not None
            continue
        if not on:
            continue
        m = re.match(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", line)
        if m:
            out.append((int(m.group(3), 16), m.group(1), m.group(2)))
    return out


def group_of(mn):
    for g, rx in GROUPS:
        if re.search(rx, mn):
            return g
    return "other"


def norm(mn):
    return re.sub(r"_e(32|64)$|_sdwa$", "", mn)


def loops_of(insts):
    """[(kind, Counter of mnemonics)] of every loop body (a backward branch)"""
    addr = {a: i for i, (a, _, _) in enumerate(insts)}
    out = []
    for i, (a, mn, ops) in enumerate(insts):
        if not (mn.startswith("s_cbranch") or mn == "s_branch"):
            continue
        off = re.match(r"(\d+)", ops)
        if not off:
            continue
        simm = int(off.group(1))
        simm = simm - 65536 if simm >= 32768 else simm
        tgt = a + 4 + 4 * simm
        if tgt < a and tgt in addr:
            body = collections.Counter(norm(m) for _, m, _ in insts[addr[tgt]:i + 1])
            out.append(body)
    return out


def classify(body):
    g = collections.Counter()
    for mn, n in body.items():
        g[group_of(mn)] += n
    return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--obj", default=os.path.join(ROOT, "linea_stark_prover_amd", "_build", "k_hash.o"))
    ap.add_argument("--kernel", default="k_merkle_level")
    ap.add_argument("--json", default=None)
    ap.add_argument("--measured-valu-per-perm", type=float, default=44069.0,
                    help="SQ_INSTS_VALU per permutation from the PMC pass (profiles/r02k_pmc_dispatch.txt)")
    a = ap.parse_args()
    asm = disassemble(a.obj)
    insts = kernel_insts(asm, a.kernel + r"ILj11ELi1E")
    if not insts:
        sys.exit(f"kernel {a.kernel}<11, 1> not found")
    bodies = loops_of(insts)
    full = [b for b in bodies if b[MAD] == 3 * 702]
    part = [b for b in bodies if b[MAD] == 702]
    if not full or not part:
        sys.exit("round loops not found (their MAD counts changed?)")
    F = min(full, key=lambda b: sum(b.values()))
    Pm = min(part, key=lambda b: sum(b.values()))
    PM = max(part, key=lambda b: sum(b.values()))
    perm = collections.Counter()
    for mn, n in F.items():
        perm[mn] += 8 * n
    for mn, n in Pm.items():
        perm[mn] += 22 * n
    groups = classify(perm)
    mem = ("LDS", "global / buffer memory", "scalar")
    valu = sum(n for g, n in groups.items() if g not in mem)
    valu_hi = valu + 22 * (sum(v for k, v in classify(PM).items() if k not in mem)
                          - sum(v for k, v in classify(Pm).items() if k not in mem))
    prods = 46 * 5
    # cycles per wave64 instruction per SIMD (profiles/r02_rates.json): 64-bit integer 4, other VALU 2.3
    cyc = {"mad (products)": 4.0, "limb split / carry: 64-bit shift": 4.0}
    rows = []
    tot_cyc = sum(n * cyc.get(g, 2.3) for g, n in groups.items() if g not in mem)
    for g, _ in GROUPS:
        n = groups.get(g, 0)
        if not n:
            continue
        r = {"group": g, "instructions_per_perm": n, "per_product": round(n / prods, 2)}
        if g not in mem:
            r["share_of_valu_instructions"] = round(n / valu, 4)
            r["share_of_valu_cycles"] = round(n * cyc.get(g, 2.3) / tot_cyc, 4)
        rows.append(r)
    res = {"kernel": f"{a.kernel}<11u, 1> (one state per lane, x^11, default layers)",
           "full_round_body": {"instructions": sum(F.values()), "mads": F[MAD], "groups": dict(classify(F))},
           "partial_round_body": {"instructions": [sum(Pm.values()), sum(PM.values())], "mads": Pm[MAD],
                                  "groups": dict(classify(Pm))},
           "valu_per_permutation_rounds": [valu, valu_hi],
           "valu_per_permutation_measured": a.measured_valu_per_perm,
           "mads_per_permutation": perm[MAD], "groups": rows, "products_per_permutation": prods,
           "method": "tools/isa_budget.py: llvm-objdump of the shipped k_hash.o; the full-round loop body (2106 MADs) "
                     "x 8 + the partial-round body (702 MADs) x 22; the compiler keeps two partial-round bodies "
                     "(both counted as bounds); the rest of the measured SQ_INSTS_VALU is the sponge / conversions"}
    print(f"{res['kernel']}")
    print(f"  full round body {sum(F.values())} instructions ({F[MAD]} MADs); partial round body "
          f"{sum(Pm.values())}..{sum(PM.values())} ({Pm[MAD]} MADs)")
    print(f"  rounds: {valu}..{valu_hi} VALU instructions per permutation ({perm[MAD]} MADs); measured "
          f"SQ_INSTS_VALU {a.measured_valu_per_perm:.0f}")
    for r in rows:
        extra = (f"  {100 * r['share_of_valu_instructions']:5.1f}% of VALU instr, {100 * r['share_of_valu_cycles']:5.1f}% "
                 f"of VALU cycles") if "share_of_valu_instructions" in r else ""
        print(f"  {r['group']:38s} {r['instructions_per_perm']:7d}  {r['per_product']:7.2f}/product{extra}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
