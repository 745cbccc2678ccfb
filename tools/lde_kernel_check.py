"""The bench's roofline kernel against the rocprofv3 kernel trace of the same
command: per launch shape of k_ntt_rm (kernel, grid), every call's duration,
and the trace LDE's per-call sum (the 2^19 x 8 LDE = the three launches with
the trace's grids) beside bench.py's live HIP-event figure (roofline.ms).

    python tools/lde_kernel_check.py <kernel_trace.csv> <bench line json> [tag]
"""
import collections
import csv
import json
import sys


def main():
    trace, line = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else ""
    calls = collections.defaultdict(list)
    for r in csv.DictReader(open(trace)):
        name = r["Kernel_Name"].replace("lsp::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if not name.startswith("k_ntt_rm"):
            continue
        grid = int(r["Grid_Size_X"])
        calls[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"The bench's roofline kernel (coset_lde_batch of the 2^19 x 8 trace = 3 launches of k_ntt_rm) against the "
          f"rocprofv3 kernel trace of the same command{(' (' + tag + ')') if tag else ''}.")
    print("The trace LDE's launches have the larger grid of each kernel; the quotient LDE's (4 columns) half of it.\n")
    trace_shapes = {}
    for (name, grid), ts in sorted(calls.items()):
        last = ts[-3:]
        print(f"{name:22s} grid {grid:8d}: {len(ts)} calls, mean {sum(ts) / len(ts):8.1f} us, "
              f"last 3 {sum(last) / len(last):8.1f} us  {[round(t, 1) for t in ts]}")
        if grid >= trace_shapes.get(name, (0, None))[0]:
            trace_shapes[name] = (grid, ts)
    n = min(len(ts) for _, ts in trace_shapes.values())
    per_call = [sum(ts[i] for _, ts in trace_shapes.values()) / 1e3 for i in range(n)]
    last = per_call[-3:]
    d = json.loads([x for x in open(line) if x.startswith("{")][-1])
    print(f"\ntrace LDE per call: {sum(per_call) / n:.3f} ms mean of {n}, {sum(last) / len(last):.3f} ms mean of the "
          f"last 3 (clocks settled)")
    print(f"bench.py's live HIP-event figure in that profiled run: roofline.ms {d['roofline']['ms']:.3f} "
          f"(lib {d.get('lib_src_sha16')})")


if __name__ == "__main__":
    main()
