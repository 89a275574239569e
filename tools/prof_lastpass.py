"""Per-kernel average durations of bench.py's kernel-timing pass, from a rocprofv3 kernel
trace of the same bench command.

bench.py runs its timed steps (two streams) and then ONE serialised step with hipEvents
around every launch; that step's dispatches are the last `per_step` of each per-plane
kernel in the trace.  This prints their rocprof average next to the overall average so the
`roofline.avg_us` of the bench line can be checked against the profiler.
usage: python tools/prof_lastpass.py KERNEL_TRACE_CSV --per-step D [--group G] [--out FILE]
"""
import argparse
import csv
import json
from collections import defaultdict

from pmc_summarize import short

GROUPED = {"cost_x", "omega_conv", "omega_stats1", "omega_stats2"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--per-step", type=int, required=True, help="launches per kernel per step (D)")
    ap.add_argument("--group", type=int, default=16,
                    help="planes per cost-stage launch (the sweep's plane group)")
    ap.add_argument("--out")
    args = ap.parse_args()
    runs = defaultdict(list)
    with open(args.trace) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            k = short(name)
            if k is None and "deconv" in name:
                k = "deconv"
            if k is None:
                continue
            runs[k].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    out = {}
    for k, v in sorted(runs.items()):
        v.sort()
        durs = [(e - s) / 1e3 for s, e in v]
        # the cost-slice kernels launch once per plane group, the regulariser's once per plane
        per = -(-args.per_step // args.group) if k in GROUPED else args.per_step
        last = durs[-per:] if len(durs) >= per else durs
        out[k] = dict(calls=len(durs), avg_us_all=round(sum(durs) / len(durs), 2),
                      avg_us_timing_pass=round(sum(last) / len(last), 2), timing_pass_calls=len(last))
        print(f"{k:14s} calls {len(durs):6d}  avg(all) {out[k]['avg_us_all']:9.2f} us  "
              f"avg(timing pass, last {len(last)}) {out[k]['avg_us_timing_pass']:9.2f} us")
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
