"""Per (kernel, grid size) summary of tools/pmc_cmd.sh passes: the same
wave-time split and per-wave instruction counts as pmc_cmd_summary.py, but
launches of one kernel with different grids (e.g. the trace and the quotient
leaf hashing) are kept apart.  Usage: python tools/pmc_dispatch_summary.py <dir>"""
import collections
import csv
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
calls = collections.defaultdict(set)
for p in ("p1", "p2"):
    for r in csv.DictReader(open(f"{root}/{p}/run_counter_collection.csv")):
        name = r["Kernel_Name"].replace("lsp::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        key = (name, int(r["Grid_Size"]))
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        if p == "p1" and r["Counter_Name"] == "SQ_WAVES":
            dur[key] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            calls[key].add(r["Dispatch_Id"])
for key, c in sorted(agg.items(), key=lambda x: -dur[x[0]]):
    if dur[key] < 1e-3:
        continue
    wc = c["SQ_WAVE_CYCLES"] or 1
    w = c["SQ_WAVES"] or 1
    clk = c["GRBM_GUI_ACTIVE"] / 8 / dur[key] / 1e9
    n = len(calls[key]) or 1
    print(f"{key[0][:34]:34s} grid {key[1]:>9d} x{n:<3d} {dur[key] / n * 1e3:8.3f} ms/call clk {clk:4.2f} | "
          f"active {c['SQ_ACTIVE_INST_ANY'] / wc:5.2f} valu {c['SQ_ACTIVE_INST_VALU'] / wc:5.2f} "
          f"wait {c['SQ_WAIT_ANY'] / wc:5.2f} stall {c['SQ_WAIT_INST_ANY'] / wc:5.2f} | per wave: valu "
          f"{c['SQ_INSTS_VALU'] / w:8.0f} lds {c['SQ_INSTS_LDS'] / w:6.0f} vmem {c['SQ_INSTS_VMEM_RD'] / w:5.0f}")
