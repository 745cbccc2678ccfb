"""Check the bench's event-timed coset_lde_batch (roofline.ms) against the
rocprofv3 kernel trace of the same LDE (tools/pmc_round.sh 'kt' pass over
tools/lde_probe.py, 3 calls): per-call sum of the LDE kernels.

    python tools/lde_agreement.py <kernel_stats.csv> <bench.json> [calls] [logcw]
"""
import csv, json, sys

stats, bench = sys.argv[1], sys.argv[2]
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 3
rows = list(csv.DictReader(open(stats)))
# which k_ntt_rm<DIF, MODE, LOGCW> instantiations belong to the LDE measured: "all" (the
# probe runs only the trace LDE; since round 2 its passes use LOGCW 0 and 1), or one LOGCW
# (round 1's bench trace: LOGCW 3 for the trace LDE, 2 for the quotient's)
logcw = sys.argv[4] if len(sys.argv) > 4 else "all"
lines, tot = [], 0.0
for r in rows:
    name = r["Name"].replace("lsp::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    targs = name[name.find("<") + 1:-1].split(", ") if "<" in name else []
    # k_ntt_rm<DIF, MODE, LOGCW> (older traces: k_ntt_rm<DIF, MODE>)
    ntt = "k_ntt_rm" in name and (logcw == "all" or len(targs) == 2 or targs[-1] == logcw)
    if ntt or "k_pow_tables" in name:
        ms = float(r["TotalDurationNs"]) / calls / 1e6
        tot += ms
        lines.append(f"  {name:28s} calls {int(r['Calls']):3d}  avg {float(r['AverageNs']) / 1e3:9.1f} us  per LDE call {ms:7.3f} ms")
b = json.load(open(bench))["roofline"]
print("coset_lde_batch (trace, 2^19 x 8 -> 2^22 x 8): rocprofv3 kernel time vs the bench's HIP-event phase")
print("\n".join(lines))
print(f"  sum per call (rocprofv3)       {tot:.3f} ms   (k_pow_tables also counts the one-off twiddle tables)")
print(f"  bench roofline.ms (HIP events)  {b['ms']:.3f} ms   achieved {b['achieved']:.1f} GB/s of {b['peak']:.0f}")
print(f"  ratio                           {b['ms'] / tot:.3f}")
