"""Per-proof GPU timeline from a rocprofv3 kernel trace: busy time, idle gaps
and the largest gaps (the host's share of the critical path).
Usage: python tools/trace_gaps.py <kernel_trace.csv> [first-kernel-substring]"""
import csv
import sys

path = sys.argv[1]
mark = sys.argv[2] if len(sys.argv) > 2 else "k_open_denoms"  # once per proof
def short(n):
    return n.replace("void ", "").replace("lsp::(anonymous namespace)::", "").replace("lsp::", "").split("(")[0][:40]


rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
# one proof period: between the last two launches of a once-per-proof kernel
a, b = starts[-2], starts[-1]
R = rows[a:b]
t0, t1 = int(R[0]["Start_Timestamp"]), int(R[-1]["End_Timestamp"])
busy, gaps, prev = 0.0, [], None
for r in R:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev is not None and s > prev[0]:
        gaps.append(((s - prev[0]) / 1e3, prev[1], short(r["Kernel_Name"]), (s - t0) / 1e6))
    busy += (e - s) / 1e3
    prev = (max(e, prev[0]) if prev else e, short(r["Kernel_Name"]))
span = (t1 - t0) / 1e3
print(f"span {span / 1e3:.2f} ms, kernels busy {busy / 1e3:.2f} ms, idle {sum(g[0] for g in gaps) / 1e3:.2f} ms")
big = sorted(gaps, reverse=True)
print(f"gaps > 20 us: {sum(1 for g in gaps if g[0] > 20)}, total {sum(g[0] for g in gaps if g[0] > 20) / 1e3:.2f} ms")
for g, x, y, at in big[:14]:
    print(f"  {g:8.1f} us at {at:7.3f} ms  after {x:40s} before {y}")
