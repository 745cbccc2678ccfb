"""Per-kernel summary of tools/pmc_cmd.sh passes: wave-time split, VALU / LDS
instructions per wave, effective clock.  SQ_*_CYCLES count quad-cycles
(MI355X_MICROARCH.md); ratios between them are unit-free."""
import collections, csv, sys
root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
for p in ("p1", "p2"):
    for r in csv.DictReader(open(f"{root}/{p}/run_counter_collection.csv")):
        name = r["Kernel_Name"].replace("lsp::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        if p == "p1" and r["Counter_Name"] == "SQ_WAVES":
            dur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
for name, c in sorted(agg.items(), key=lambda x: -dur[x[0]]):
    if dur[name] < 1e-4:
        continue
    wc = c["SQ_WAVE_CYCLES"] or 1
    w = c["SQ_WAVES"] or 1
    clk = c["GRBM_GUI_ACTIVE"] / 8 / dur[name] / 1e9
    print(f"{name[:48]:48s} {dur[name]*1e3:8.2f} ms clk {clk:4.2f} | active {c['SQ_ACTIVE_INST_ANY']/wc:5.2f} "
          f"valu {c['SQ_ACTIVE_INST_VALU']/wc:5.2f} wait {c['SQ_WAIT_ANY']/wc:5.2f} stall {c['SQ_WAIT_INST_ANY']/wc:5.2f} "
          f"ldsstall {c['SQ_WAIT_INST_LDS']/wc:5.2f} | per wave: valu {c['SQ_INSTS_VALU']/w:8.0f} lds {c['SQ_INSTS_LDS']/w:6.0f} "
          f"vmem {c['SQ_INSTS_VMEM_RD']/w:5.0f} salu {c['SQ_INSTS_SALU']/w:5.0f} bankconf/lds {c['SQ_LDS_BANK_CONFLICT']/max(1,c['SQ_INSTS_LDS']):.2f}")
