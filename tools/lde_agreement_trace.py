"""The bench's event-timed trace LDE (roofline.ms, the last timed step) against
the rocprofv3 kernel trace of the same command (tools/gpu.sh 'rocprof'
step): per proof, the trace LDE is the first three k_ntt_rm dispatches (inverse
pass, fused pass, in-place pass; the quotient LDE's three follow).

    python tools/lde_agreement_trace.py <bench_kernel_trace.csv> <prof_bench.json>
"""
import csv
import json
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ntt = [r for r in rows if "k_ntt_rm" in r["Kernel_Name"]]
groups = [ntt[i:i + 6] for i in range(0, len(ntt) - len(ntt) % 6, 6)]
print("trace coset_lde_batch (2^19 x 8 -> 2^22 x 8) per proof: rocprofv3 kernel time vs the bench's HIP events")
for i, g in enumerate(groups):
    parts = [(x["Kernel_Name"].replace("void ", "").replace("lsp::(anonymous namespace)::", "").split("(")[0],
              (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3) for x in g[:3]]
    tot = sum(us for _, us in parts) / 1e3
    print(f"  proof {i}: {tot:.3f} ms  = " + " + ".join(f"{n} {us:.1f} us" for n, us in parts))
b = json.load(open(sys.argv[2]))["roofline"]
last = sum((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) for x in groups[-1][:3]) / 1e6
print(f"  bench roofline.ms (HIP events, last timed step) {b['ms']:.3f} ms; last proof's kernels {last:.3f} ms; "
      f"ratio {b['ms'] / last:.3f}")
print("  (the first proofs are the bench's warm-up steps, at a clock still ramping)")
