#!/bin/bash
# A/B of library builds on the headline sweep (cells' per-kernel times from bench.py's timing
# pass): bash tools/cell_ab.sh TAG lib1 lib2 ... ("default" = the in-tree library)
set -u
TAG=$1; shift
mkdir -p gpurun_out
for lib in "$@"; do
  if [ "$lib" = default ]; then unset AARMVS_LIB; else export AARMVS_LIB=$lib; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --no-fusion --no-train --steps 3 --warmup 1 > gpurun_out/${TAG}_$(basename $lib .so).log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); k=d['kernels']; print(sys.argv[2], round(d['value']/1e9,4), {n: k[n]['avg_us'] for n in k if n.startswith('lstm')})" gpurun_out/${TAG}_$(basename $lib .so).log $lib | tee -a gpurun_out/${TAG}_ab.txt
done
