"""Per (kernel variant, grid) average durations of the k_ntt_rm launches in a
rocprofv3 kernel trace (tools/time_lde.py under --kernel-trace)."""
import collections, csv, sys
agg = collections.defaultdict(lambda: [0, 0.0, 0])
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "k_ntt" not in n:
        continue
    k = (n.split("<")[1].split(">")[0], int(r["Grid_Size_X"]), int(r["LDS_Block_Size"]))
    a = agg[k]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a[2] = int(r["VGPR_Count"])
for k, (c, t, vg) in sorted(agg.items()):
    print(f"{k[0]:12s} grid {k[1]:9d} lds {k[2]:6d} calls {c:4d} avg {t / c:9.1f} us vgpr {vg}")
