"""Print the per-dispatch timeline of the last full engine step in a rocprofv3
kernel trace (tools/kernel_trace.sh output)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ktrace/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "append_samples_kernel" in r["Kernel_Name"]]
s, e = starts[-2], starts[-1]
prev = None
tot = {}
for r in rows[s:e]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("void ", "").replace("vamd::", "").split("(")[0]
    gap = (st - prev) / 1e3 if prev else 0.0
    print(f"{name:34s} grid={int(r['Grid_Size_X'])//int(r['Workgroup_Size_X']):5d}x{r['Grid_Size_Y']:>3s} "
          f"wg={r['Workgroup_Size_X']:>4s} vgpr={r['VGPR_Count']:>3s} lds={r['LDS_Block_Size']:>6s} "
          f"dur={(en - st) / 1e3:8.1f}us gap={gap:6.1f}us")
    tot[name] = tot.get(name, 0) + (en - st) / 1e3
    prev = en
print("step span us:", (int(rows[e]["Start_Timestamp"]) - int(rows[s]["Start_Timestamp"])) / 1e3)
for k, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {k:34s} {v:9.1f}us")
