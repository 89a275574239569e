"""Per-kernel table of a rocprofv3 kernel_stats.csv: python tools/prof_table.py CSV [PLANES] [N]
(PLANES: planes the profiled program swept, to print microseconds per plane)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
planes = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = [r for r in rows if "aarmvs" in r["Name"] or len(sys.argv) > 4]
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.3f} ms = {tot / 1e3 / planes:.1f} us/plane")
for r in rows[:n]:
    print(f"{r['Name'][:64]:64s} {int(r['Calls']):6d} {float(r['TotalDurationNs']) / 1e3 / planes:9.1f} "
          f"us/plane  avg {float(r['AverageNs']) / 1e3:9.1f} us")
