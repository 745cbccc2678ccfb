"""Summarize a rocprofv3 kernel_stats.csv (per-proof figures for N proves)."""
import csv, sys
path = sys.argv[1]; nproves = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"{'kernel':64s} {'calls':>7s} {'avg_us':>9s} {'ms/proof':>9s} {'pct':>6s}")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
    name = r['Name'].replace('lsp::(anonymous namespace)::', '').replace('void ', '')[:64]
    print(f"{name:64s} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.1f} {float(r['TotalDurationNs'])/1e6/nproves:9.2f} {float(r['Percentage']):6.1f}")
print(f"total kernel time per proof: {tot/1e6/nproves:.2f} ms")
