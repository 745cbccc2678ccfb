"""Per-kernel VALU/LDS counter summary from tools/pmc_valu.sh passes.

VALU issue utilisation = SQ_INSTS_VALU x 4 cycles (one wave64 VALU op per 4
cycles per SIMD) / (1024 SIMDs x kernel cycles), kernel cycles from
GRBM_GUI_ACTIVE / 8 XCDs (MI355X_MICROARCH.md, DVFS note) -- the share of
the chip's VALU issue slots the kernel used.  Also: effective clock,
SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of wave time issuing VALU),
LDS wait share and bank conflicts per LDS instruction."""
import collections, csv, os, sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
calls = collections.Counter()
for p in ("p1", "p2", "p3"):
    seen = set()
    path = f"{root}/{p}/run_counter_collection.csv"
    if p != "p1" and not os.path.exists(path):  # tools/box_clock.sh runs no LDS pass
        continue
    for r in csv.DictReader(open(path)):
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
    util = c["SQ_INSTS_VALU"] * 4 / (1024 * cyc) if cyc else 0  # every instruction at 4 cycles (upper bound)
    # class-weighted (profiles/r02_rates.json): 64-bit integer ops (v_mad_u64_u32,
    # 64-bit shifts/adds) 4 cycles per wave64 per SIMD, other VALU >= 2 -- a lower bound
    i64 = c.get("SQ_INSTS_VALU_INT64", 0.0)
    util_lb = (4 * i64 + 2 * (c["SQ_INSTS_VALU"] - i64)) / (1024 * cyc) if cyc else 0
    # SIMD VALU busy: every wave's VALU-issue cycles (SQ_ACTIVE_INST_VALU, quad-cycles)
    # summed, over the chip's SIMD-cycles
    busy = 4 * c["SQ_ACTIVE_INST_VALU"] / (1024 * cyc) if cyc else 0
    act = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"] if c["SQ_WAVE_CYCLES"] else 0
    ldsw = c["SQ_WAIT_INST_LDS"] / c["SQ_WAVE_CYCLES"] if c["SQ_WAVE_CYCLES"] else 0
    bc = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"] if c["SQ_INSTS_LDS"] else 0
    rows.append((dur[name], name, calls[name], clk, util, act, ldsw, bc, c["SQ_INSTS_VALU"] / max(c["SQ_WAVES"], 1),
                 util_lb, busy))
rows.sort(reverse=True)
if len(sys.argv) > 2:  # JSON for bench.py (profiles/*_valu_pmc.json)
    import json
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from linea_stark_prover_amd.build import library_hash, source_hash
    stamp = os.path.join(os.path.dirname(os.path.abspath(root)), "lib_src_sha16.txt")
    json.dump({"lib_src_sha16": open(stamp).read().strip() if os.path.exists(stamp) else (library_hash() or source_hash()),
               "method": "rocprofv3 --pmc passes (tools/pmc_valu.sh) over tools/time_prove.py 19; "
                         "valu_issue = SQ_ACTIVE_INST_VALU x 4 (all waves) / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): "
                         "the share of SIMD cycles issuing VALU; valu_issue_x4 = SQ_INSTS_VALU x 4 / (same) "
                         "(every instruction at the MAD's 4 cycles, r01's measure, reads > 1 for 2-cycle-heavy "
                         "kernels); valu_issue_lb = class-weighted (INT64 x 4 + other x 2)",
               "kernels": {name: {"calls": n, "ms": d * 1e3, "clock_ghz": clk, "valu_issue": busy,
                                  "valu_issue_x4": util, "valu_issue_lb": ulb,
                                  "valu_active_per_wave": act, "lds_wait": ldsw, "lds_bank_conflicts_per_inst": bc}
                           for d, name, n, clk, util, act, ldsw, bc, vpw, ulb, busy in rows}},
              open(sys.argv[2], "w"), indent=1)
print(f"{'kernel':34s} {'calls':>5s} {'ms':>8s} {'GHz':>5s} {'VALUbusy':>8s} {'issue_x4':>8s} {'issue_lb':>8s} {'valu/wave':>9s} {'ldswait':>7s} {'bankc/lds':>9s} {'valu/wave#':>10s}")
for d, name, n, clk, util, act, ldsw, bc, vpw, ulb, busy in rows:
    print(f"{name[:34]:34s} {n:5d} {d * 1e3:8.2f} {clk:5.2f} {busy:8.2f} {util:8.2f} {ulb:8.2f} {act:9.2f} {ldsw:7.2f} {bc:9.2f} {vpw:10.0f}")
