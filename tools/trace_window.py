"""Kernels of one proof between two marker kernels, with start / end relative
to the first marker (diagnostic for overlapping streams).
Usage: python tools/trace_window.py <kernel_trace.csv> <from-substring> <to-substring> [nth-proof]
e.g. the trace tree's narrow levels and the side stream's constraint evaluation:
    python tools/trace_window.py trace.csv k_hash_rows1 k_quotient_fold 2"""
import csv
import sys


def short(n):
    return n.replace("void ", "").replace("lsp::(anonymous namespace)::", "").replace("lsp::", "").split("(")[0][:44]


path, a, b = sys.argv[1], sys.argv[2], sys.argv[3]
nth = int(sys.argv[4]) if len(sys.argv) > 4 else 1
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if a in r["Kernel_Name"]]
i0 = starts[min(nth, len(starts) - 1)] if nth < len(starts) else starts[-1]
i1 = next(i for i in range(i0, len(rows)) if b in rows[i]["Kernel_Name"])
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} us  q{r.get('Queue_Id', '?'):>3s}  "
          f"{short(r['Kernel_Name'])}")
