"""GPU busy time of a rocprofv3 kernel trace (``--kernel-trace --output-format csv``) over the
last STEPS steps of a ``bench.py --train`` run: the union of all kernel intervals (streams
overlap), the idle time between them, the largest idle gaps with the kernels on either side, and
a timeline in BIN_MS bins (busy fraction and the category holding most kernel time in the bin:
F forward sweep, B backward sweep, O everything else -- FeatNet, loss, optimizer, copies).
usage: python tools/trace_busy.py TRACE.csv STEP_MS [STEPS] [BIN_MS]"""
import csv
import sys

BWD = ("bwd", "dgrad", "wgrad", "cbw", "grad", "gnb", "fold", "bptt", "backward")
FWD = ("omega", "cost_x", "stat_reduce", "lstm_cell", "deconv_mfma", "head_wta", "to_c8", "finalize")


def category(name: str) -> str:
    n = name.lower()
    if "aarmvs" not in n and not any(k in n for k in FWD + BWD):
        return "O"
    if any(k in n for k in BWD):
        return "B"
    if any(k in n for k in FWD):
        return "F"
    return "O"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    step_ms = float(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    bin_ms = float(sys.argv[4]) if len(sys.argv) > 4 else 5.0
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    t_end = max(e for _, e, _ in iv)
    t0 = t_end - steps * step_ms * 1e6
    iv = [(max(s, t0), e, n) for s, e, n in iv if e > t0]
    busy, gaps = 0.0, []
    cur_s, cur_e, last = iv[0][0], iv[0][1], iv[0][2]
    for s, e, n in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, last, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        if e >= cur_e:
            last = n
    busy += cur_e - cur_s
    span = t_end - t0
    print(f"window {span / 1e6:.1f} ms ({steps} steps): busy {busy / 1e6:.1f} ms "
          f"({busy / span:.1%}), idle {(span - busy) / 1e6:.1f} ms per window")
    gaps.sort(reverse=True)
    print("largest idle gaps (us, after -> before):")
    for g, a, b in gaps[:15]:
        print(f"  {g / 1e3:8.1f}  {a[:60]} -> {b[:60]}")
    small = sum(g for g, _, _ in gaps if g < 20e3)
    print(f"gaps under 20 us: {len([g for g, _, _ in gaps if g < 20e3])}, {small / 1e6:.2f} ms")
    nb = int(span / (bin_ms * 1e6)) + 1
    occ = [0.0] * nb
    cat = [dict(F=0.0, B=0.0, O=0.0) for _ in range(nb)]
    for s, e, n in iv:
        c = category(n)
        b = int((s - t0) / (bin_ms * 1e6))
        while s < e and b < nb:
            be = t0 + (b + 1) * bin_ms * 1e6
            d = min(e, be) - s
            cat[b][c] += d
            s = min(e, be)
            b += 1
    # busy per bin from the merged union
    merged = []
    for s, e, _ in iv:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    for s, e in merged:
        b = int((s - t0) / (bin_ms * 1e6))
        while s < e and b < nb:
            be = t0 + (b + 1) * bin_ms * 1e6
            occ[b] += min(e, be) - s
            s = min(e, be)
            b += 1
    line = []
    for b in range(nb):
        f = occ[b] / (bin_ms * 1e6)
        c = max(cat[b], key=cat[b].get) if sum(cat[b].values()) else "."
        line.append(f"{c}{min(9, int(f * 10))}")
    print(f"timeline, {bin_ms:g} ms bins (category, busy tenths):")
    for i in range(0, nb, 20):
        print("  " + " ".join(line[i:i + 20]))


if __name__ == "__main__":
    main()
