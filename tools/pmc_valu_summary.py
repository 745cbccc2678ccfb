"""Per-kernel VALU/LDS counter summary from tools/pmc_valu.sh passes.

VALU issue utilisation = SQ_INSTS_VALU x 4 cycles (one wave64 VALU op per 4
cycles per SIMD) / (1024 SIMDs x kernel cycles), kernel cycles from
GRBM_GUI_ACTIVE / 8 XCDs (MI355X_MICROARCH.md, DVFS note) -- the share of
the chip's VALU issue slots the kernel used.  Also: effective clock,
SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of wave time issuing VALU),
LDS wait share and bank conflicts per LDS instruction."""
import collections, csv, sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
calls = collections.Counter()
for p in ("p1", "p2", "p3"):
    seen = set()
    for r in csv.DictReader(open(f"{root}/{p}/run_counter_collection.csv")):
        name = r["Kernel_Name"].replace("lsp::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (r["Dispatch_Id"], p)
        if p == "p1" and key not in seen:
            seen.add(key)
            dur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            calls[name] += 1
rows = []
for name, c in agg.items():
    if dur[name] < 1e-4 or "copyBuffer" in name:
        continue
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    clk = cyc / dur[name] / 1e9 if dur[name] else 0
    util = c["SQ_INSTS_VALU"] * 4 / (1024 * cyc) if cyc else 0
    act = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"] if c["SQ_WAVE_CYCLES"] else 0
    ldsw = c["SQ_WAIT_INST_LDS"] / c["SQ_WAVE_CYCLES"] if c["SQ_WAVE_CYCLES"] else 0
    bc = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"] if c["SQ_INSTS_LDS"] else 0
    rows.append((dur[name], name, calls[name], clk, util, act, ldsw, bc, c["SQ_INSTS_VALU"] / max(c["SQ_WAVES"], 1)))
rows.sort(reverse=True)
if len(sys.argv) > 2:  # JSON for bench.py (profiles/*_valu_pmc.json)
    import json
    json.dump({"method": "rocprofv3 --pmc passes (tools/pmc_valu.sh) over tools/time_prove.py 19; "
                         "valu_issue = SQ_INSTS_VALU * 4 / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)",
               "kernels": {name: {"calls": n, "ms": d * 1e3, "clock_ghz": clk, "valu_issue": util,
                                  "valu_active_per_wave": act, "lds_wait": ldsw, "lds_bank_conflicts_per_inst": bc}
                           for d, name, n, clk, util, act, ldsw, bc, vpw in rows}},
              open(sys.argv[2], "w"), indent=1)
print(f"{'kernel':34s} {'calls':>5s} {'ms':>8s} {'GHz':>5s} {'VALUissue':>9s} {'valu/wave':>9s} {'ldswait':>7s} {'bankc/lds':>9s} {'valu/wave#':>10s}")
for d, name, n, clk, util, act, ldsw, bc, vpw in rows:
    print(f"{name[:34]:34s} {n:5d} {d * 1e3:8.2f} {clk:5.2f} {util:9.2f} {act:9.2f} {ldsw:7.2f} {bc:9.2f} {vpw:10.0f}")
