"""Per-kernel ceiling table from tools/gpu_ceiling.sh's PMC passes (one 16-plane group of the
headline sweep): python tools/ceiling_summary.py DIR [--out FILE]

For each kernel (cost-slice kernels and cells): waves, wave-cycles split into issuing /
waiting on a dependency / parked (s_waitcnt, barrier), instruction mix per wave, LDS bank
conflicts, TA busy (fraction of GRBM_GUI_ACTIVE), L1 (TCP) accesses and L1->L2 requests,
L2 hit rate, HBM bytes (FETCH_SIZE doubled per the gfx950 correction, + WRITE_SIZE).
Busy fractions are per unit over the kernel's active cycles (GRBM_GUI_ACTIVE / 8 XCDs); TD is
averaged over the 256 CUs' units."""
import argparse
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summarize import short  # noqa: E402


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Dispatch_Id"]
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            name[k] = r["Kernel_Name"]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for k, cs in per.items():
        for c, v in cs.items():
            agg[short(name[k])][c].append(v)
    return {n: {c: sum(v) / len(v) for c, v in cs.items()} for n, cs in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    ap.add_argument("--kernels", default="omega_conv,cost_x,omega_stats1,omega_stats2,lstm_cell0,lstm_cell4")
    args = ap.parse_args()
    passes = ["sq_time", "sq_mix", "tex", "l2", "fetch", "write"]
    if os.path.isdir(os.path.join(args.dir, "f64")):
        passes.append("f64")
    P = {p: load(os.path.join(args.dir, p)) for p in passes}
    kernels = args.kernels.split(",")
    res = {}
    for k in kernels:
        g = lambda p, c: P[p].get(k, {}).get(c)  # noqa: E731
        r = {}
        wc = g("sq_time", "SQ_WAVE_CYCLES")
        if wc:
            r["waves"] = g("sq_time", "SQ_WAVES")
            r["issue_frac"] = g("sq_time", "SQ_ACTIVE_INST_ANY") / wc
            r["dep_stall_frac"] = g("sq_time", "SQ_WAIT_INST_ANY") / wc
            r["lds_issue_stall_frac"] = g("sq_time", "SQ_WAIT_INST_LDS") / wc
            r["parked_frac"] = g("sq_time", "SQ_WAIT_ANY") / wc
            r["vmem_issue_frac"] = g("sq_time", "SQ_ACTIVE_INST_VMEM") / wc
        waves = r.get("waves")
        if waves and g("sq_mix", "SQ_INSTS_VALU") is not None:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_MFMA",
                      "SQ_INSTS_SALU"):
                r[c.lower().replace("sq_insts_", "per_wave_")] = g("sq_mix", c) / waves
            lds = g("sq_mix", "SQ_LDS_IDX_ACTIVE")
            r["lds_bank_conflict_frac"] = g("sq_mix", "SQ_LDS_BANK_CONFLICT") / lds if lds else None
        gui = g("tex", "GRBM_GUI_ACTIVE")
        if gui:
            gui /= 8.0   # rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs (MI355X_MICROARCH.md)
            r["ta_busy_frac"] = g("tex", "TA_BUSY_avr") / gui
            r["td_busy_frac"] = g("tex", "TD_TD_BUSY_sum") / gui / 256.0
            r["tcp_accesses"] = g("tex", "TCP_TOTAL_CACHE_ACCESSES_sum")
            r["tcp_to_l2_read_req"] = g("tex", "TCP_TCC_READ_REQ_sum")
            r["ta_wavefronts"] = g("tex", "TA_TOTAL_WAVEFRONTS_sum")
            r["gui_active_cycles"] = gui
        req = g("l2", "TCC_REQ_sum")
        if req:
            r["l2_req"] = req
            r["l2_hit_frac"] = g("l2", "TCC_HIT_sum") / req
            r["l2_to_hbm_rdreq"] = g("l2", "TCC_EA0_RDREQ_sum")
        if "f64" in P and waves:
            for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                      "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_TRANS_F32"):
                v = g("f64", c)
                if v is not None:
                    r[c.lower().replace("sq_insts_valu_", "per_wave_")] = v / waves
            av, gt = g("f64", "SQ_ACTIVE_INST_VALU"), g("f64", "GRBM_GUI_ACTIVE")
            if av is not None and wc:
                r["valu_issue_frac"] = av / wc
        f, w = g("fetch", "FETCH_SIZE"), g("write", "WRITE_SIZE")
        if f is not None and w is not None:
            r["hbm_bytes_per_launch"] = (2 * f + w) * 1024
        res[k] = {a: (round(b, 4) if isinstance(b, float) else b) for a, b in r.items()}
    txt = json.dumps(res, indent=1)
    print(txt)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
