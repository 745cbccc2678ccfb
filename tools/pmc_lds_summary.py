"""Per-kernel LDS counters of one rocprofv3 --pmc pass (tools/gpu.sh pmclds:<lib>):
SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (extra LDS cycles per LDS instruction, the
figure tools/lds_banks.py models), SQ_WAIT_INST_LDS / SQ_INSTS_LDS, and the
kernel's summed duration, for every kernel above 0.1 ms in total.

    python tools/pmc_lds_summary.py <run_counter_collection.csv>
"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
seen = set()
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("lsp::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Dispatch_Id"] not in seen:
        seen.add(r["Dispatch_Id"])
        dur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
print(f"{'kernel':36s} {'ms':>8s} {'lds_instr':>12s} {'bankc/lds':>9s} {'wait/lds':>9s}")
for name in sorted(agg, key=lambda n: -dur[n]):
    c = agg[name]
    n = c.get("SQ_INSTS_LDS", 0.0)
    if dur[name] < 0.1 or n == 0:
        continue
    print(f"{name:36s} {dur[name]:8.2f} {n:12.0f} {c.get('SQ_LDS_BANK_CONFLICT', 0) / n:9.2f} "
          f"{c.get('SQ_WAIT_INST_LDS', 0) / n:9.2f}")
