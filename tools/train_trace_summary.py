"""Per-step kernel time of a rocprofv3 kernel trace of `bench.py --train` (tools/gpu_train_profile.sh):
the library's kernels against everything else (FeatNet, loss, optimizer), over the last STEPS
steps of the trace.  usage: python tools/train_trace_summary.py TRACE.csv STEP_MS [STEPS]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
step_ms = float(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
t_end = max(r["e"] for r in rows if "aarmvs" in r["Kernel_Name"])
win = [r for r in rows if r["s"] >= t_end - steps * step_ms * 1e6 and r["e"] <= t_end + 5e6]
cat, names = collections.Counter(), collections.Counter()
for r in win:
    d = (r["e"] - r["s"]) / 1e6
    c = "aarmvs" if "aarmvs" in r["Kernel_Name"] else "other"
    cat[c] += d
    names[(c, r["Kernel_Name"][:100])] += d
print({k: round(v / steps, 1) for k, v in cat.items()}, "ms of kernel time per step (streams overlap)")
for (c, n), v in names.most_common(60):
    if c != "aarmvs" and v / steps > 0.3:
        print(f"{v / steps:8.2f} ms/step  {n}")
