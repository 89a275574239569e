"""Streams and hardware queues of a rocprofv3 kernel trace (``--kernel-trace --output-format
csv``) over the WINDOW_MS ending at the last kernel whose name holds ANCHOR (default lstm_cell): per Stream_Id the Queue_Id(s) its kernels ran on, the kernel count
and busy time; the union of all kernel intervals (busy / idle); per kernel name the count and
average duration.
usage: python tools/trace_streams.py TRACE.csv WINDOW_MS [ANCHOR]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    win_ms = float(sys.argv[2])
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    anchor = sys.argv[3] if len(sys.argv) > 3 else "lstm_cell"
    t_end = max(r["e"] for r in rows if anchor in r["Kernel_Name"])
    t0 = t_end - win_ms * 1e6
    rows = [r for r in rows if r["s"] >= t0 and r["e"] <= t_end]
    per = collections.defaultdict(lambda: [set(), 0, 0.0])
    for r in rows:
        p = per[r["Stream_Id"]]
        p[0].add(r["Queue_Id"])
        p[1] += 1
        p[2] += (r["e"] - r["s"]) / 1e3
    print(f"last {win_ms:g} ms: {len(rows)} kernels")
    for sid, (qs, n, us) in sorted(per.items()):
        print(f"  stream {sid:>3}: queues {sorted(qs)}  kernels {n:6d}  busy {us / 1e3:8.2f} ms")
    iv = sorted((r["s"], r["e"]) for r in rows)
    busy, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    span = t_end - iv[0][0]
    print(f"union busy {busy / 1e6:.2f} ms of {span / 1e6:.2f} ms ({busy / span:.1%})")
    names = collections.defaultdict(list)
    for r in rows:
        names[r["Kernel_Name"].split("(")[0][:70]].append((r["e"] - r["s"]) / 1e3)
    for n, v in sorted(names.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {len(v):6d} x {sum(v) / len(v):8.2f} us = {sum(v) / 1e3:8.2f} ms  {n}")


if __name__ == "__main__":
    main()
