"""Group a rocprofv3 kernel_trace.csv by (kernel, grid, workgroup): calls, total and mean
duration.  python tools/trace_summary.py TRACE.csv OUT.csv"""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: [0, 0.0])
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        grid = "x".join(r.get(k, "") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
        wg = "x".join(r.get(k, "") for k in ("Workgroup_Size_X", "Workgroup_Size_Y", "Workgroup_Size_Z"))
        key = (r["Kernel_Name"], grid, wg, r.get("LDS_Block_Size", r.get("Lds_Size", "")),
               r.get("VGPR_Count", r.get("Arch_VGPR_Count", "")))
        a = acc[key]
        a[0] += 1
        a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
rows = sorted(acc.items(), key=lambda kv: -kv[1][1])
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "grid", "workgroup", "lds", "vgpr", "calls", "total_us", "mean_us"])
    for (name, grid, wg, lds, vg), (n, t) in rows:
        w.writerow([name[:120], grid, wg, lds, vg, n, round(t, 1), round(t / n, 2)])
