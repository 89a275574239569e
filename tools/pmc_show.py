"""Print per-kernel averages of rocprofv3 counter CSVs: python tools/pmc_show.py DIR [substr...]"""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for r in csv.DictReader(open(f)):
        d = r["Dispatch_Id"]
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        name[d] = r["Kernel_Name"]
    for d, cs in per.items():
        for k, v in cs.items():
            agg[name[d]][k].append(v)
keys = sys.argv[2:]
for n, cs in agg.items():
    if keys and not any(k in n for k in keys):
        continue
    print(n[:60])
    print("   " + "  ".join(f"{k}={sum(v) / len(v):.4g}" for k, v in sorted(cs.items())))
