"""Per-kernel HBM bytes per launch from rocprofv3 --pmc CSVs (FETCH_SIZE, WRITE_SIZE).

FETCH_SIZE/WRITE_SIZE are in KB (x1024).  gfx950 correction (MI355X_MICROARCH.md §HBM):
FETCH_SIZE reports 1/2 of the bytes of a wide (16 B/lane) coalesced stream, so the read
side is reported both raw and doubled; the doubled value is an upper bound for kernels
whose reads are not all 16-B/lane.
usage: python tools/pmc_summarize.py FETCH_DIR WRITE_DIR [--workload NAME] [--out FILE]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

SHORT = [("cost_x_kernel", "cost_x"), ("omega_conv_kernel", "omega_conv"), ("omega_mfma_kernel", "omega_conv"),
         ("omega_stats_kernel<1>", "omega_stats1"),
         ("omega_stats_kernel<2>", "omega_stats2"), ("deconv_mfma_kernel", "deconv"), ("deconv_px2_kernel", "deconv"), ("deconv_px_kernel", "deconv"), ("deconv_kernel", "deconv"), ("head_wta", "head_wta"), ("nchw_to_c8", "to_c8"), ("fusion_filter_kernel", "fusion"),
         ("cbw_feat_kernel", "cbw_feat"), ("dgrad_kernel<64>", "dgrad64"), ("dgrad_kernel<32>", "dgrad32"),
         ("wgrad2_kernel<64, 3>", "wgrad64x3"), ("wgrad2_kernel<64, 2>", "wgrad64x2"),
         ("wgrad2_kernel<32, 3>", "wgrad32x3"), ("gate_bwd_kernel", "gate_bwd"), ("cbw_chain_kernel", "cbw_chain"),
         ("deconv_wgrad_kernel", "deconv_wgrad"), ("head_wgrad_kernel", "head_wgrad"),
         ("deconv_bwd_kernel", "deconv_bwd")]


CELL = re.compile(r"lstm_cell_h3(?:db)?_kernel<(\d),")


def short(name):
    m = CELL.search(name)
    if m:
        return "lstm_cell" + m.group(1)
    for key, s in SHORT:
        if key in name:
            return s
    return None


def load(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = short(row.get("Kernel_Name", ""))
                if k:
                    vals[(k, row.get("Dispatch_Id"))].append(float(row["Counter_Value"]))
    per = defaultdict(list)
    for (k, _), v in vals.items():
        per[k].append(sum(v))   # summed over XCD / TCC instances
    return {k: sum(v) / len(v) * 1024.0 for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--workload", default="dtu_eval_1600x1184_n7_d512")
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--source", required=True,
                    help="which PMC run these are (round, command), carried into bench.py's line")
    args = ap.parse_args()
    fetch = load(args.fetch_dir, "FETCH_SIZE")
    write = load(args.write_dir, "WRITE_SIZE")
    rows = {}
    for k in sorted(set(fetch) | set(write)):
        fr, w = fetch.get(k, 0.0), write.get(k, 0.0)
        rows[k] = {"fetch_bytes_raw": fr, "fetch_bytes_x2": 2 * fr, "write_bytes": w,
                   "hbm_bytes": 2 * fr + w}
        print(f"{k:14s} fetch(raw) {fr/1e9:8.3f} GB  fetch(x2) {2*fr/1e9:8.3f} GB  "
              f"write {w/1e9:8.3f} GB per launch")
    tab = {}
    if os.path.exists(args.out):
        with open(args.out) as f:
            tab = json.load(f)
    tab[args.workload] = {k: v["hbm_bytes"] for k, v in rows.items()}
    tab.setdefault("_detail", {})[args.workload] = rows
    tab["_source"] = args.source
    with open(args.out, "w") as f:
        json.dump(tab, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
