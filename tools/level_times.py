"""Per-launch durations of the Merkle / hash kernels of one proof, grouped by
kernel and grid size, from a rocprofv3 kernel trace: where the tree time goes
level by level, and how far each level is from the throughput rate.
Usage: python tools/level_times.py <kernel_trace.csv> [perm_rate_M_per_s]"""
import collections
import csv
import sys

path = sys.argv[1]
rate = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 784.6e6
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_quotient" in r["Kernel_Name"]]
R = rows[starts[-2]:starts[-1]]  # one proof period
agg = collections.defaultdict(lambda: [0, 0.0])
for r in R:
    name = r["Kernel_Name"]
    if not any(k in name for k in ("k_merkle_level", "k_hash_rows", "k_fold_hash")):
        continue
    short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("lsp::", "")
    grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    wg = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 0)
    a = agg[(short, grid, wg)]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"{'kernel':34s} {'grid':>9s} {'wg':>4s} {'n':>3s} {'avg_us':>9s} {'sum_ms':>7s}  lanes/us")
for (k, g, w), (n, us) in sorted(agg.items(), key=lambda x: (x[0][0], -x[0][1])):
    print(f"{k:34s} {g:9d} {w:4d} {n:3d} {us / n:9.1f} {us / 1e3:7.3f}  {g / (us / n):8.0f}")
print(f"total {tot / 1e3:.2f} ms per proof; throughput floor for one-state-per-lane grids: {rate / 1e6:.0f} M lanes/s")
