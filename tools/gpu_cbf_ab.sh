#!/bin/bash
# cbw_feat ablation timing on the GPU box: per tools/ab/lib_*.so variant, the backward over one
# 16-plane group (tools/cbf_probe.py) under rocprofv3's kernel statistics.
# usage (on the box): bash tools/gpu_cbf_ab.sh name1 name2 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cbf
for n in "$@"; do
  AARMVS_LIB=$R/tools/ab/lib_$n.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/cbf/$n -o run -- \
    python3 $R/tools/cbf_probe.py > $R/gpurun_out/cbf/$n.log 2>&1 || { echo "variant $n failed"; tail -5 $R/gpurun_out/cbf/$n.log; exit 1; }
  st=$(find $R/gpurun_out/cbf/$n -name '*kernel_stats.csv' | head -1)
  echo "== $n: $(grep -h 'backward' $R/gpurun_out/cbf/$n.log)"
  python3 - "$st" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if 'cbw' in r['Name'] or 'warp_bwd' in r['Name']:
        print(f"   {r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
