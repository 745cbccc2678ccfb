"""Summarize a rocprofv3 kernel_stats.csv (per-proof figures for N proves).

Kernels that are not part of a proof -- the bench's Poseidon2 chain probe
(k_calib_perm, roofline_valu.register_resident_chain_mperm_per_s), the
trace generator and the runtime's copy kernels -- are listed apart and left
out of the per-proof total."""
import csv, sys

NOT_PROOF = ("k_calib_perm", "k_gen_perm_trace", "k_calib_")
path = sys.argv[1]; nproves = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(path)))


def clean(r):
    return r['Name'].replace('lsp::(anonymous namespace)::', '').replace('void ', '')


proof = [r for r in rows if not clean(r).startswith(NOT_PROOF)]
other = [r for r in rows if clean(r).startswith(NOT_PROOF)]
tot = sum(float(r['TotalDurationNs']) for r in proof)
print(f"{'kernel':64s} {'calls':>7s} {'avg_us':>9s} {'ms/proof':>9s} {'pct':>6s}")
for r in sorted(proof, key=lambda r: -float(r['TotalDurationNs'])):
    print(f"{clean(r)[:64]:64s} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.1f} "
          f"{float(r['TotalDurationNs'])/1e6/nproves:9.2f} {100 * float(r['TotalDurationNs']) / tot:6.1f}")
print(f"total kernel time per proof: {tot/1e6/nproves:.2f} ms (proof kernels only)")
for r in other:
    print(f"not a proof kernel, excluded: {clean(r)[:64]} {int(r['Calls'])} calls, {float(r['TotalDurationNs'])/1e6:.2f} ms")
