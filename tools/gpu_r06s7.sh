#!/bin/bash
# Round-6 cell tile shapes (AARMVS_CELL_MS): digest + headline A/B against tools/ab/lib_base.so,
# config 1 / config 2 / the training step with the old shapes (AARMVS_CELL_MS=0) and the
# per-geometry default, then the GPU suite.
set -o pipefail
T=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_r06_ab.sh $T base notests || exit 1
for ms in 0 auto; do
  if [ $ms = auto ]; then unset AARMVS_CELL_MS; else export AARMVS_CELL_MS=$ms; fi
  timeout -k 10 200 python bench.py --config plumbing_160x128_n3_d48 --steps 20 --warmup 3 --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing > gpurun_out/${T}_cfg1_ms$ms.json 2> gpurun_out/${T}_cfg1_ms$ms.err || exit 1
  timeout -k 10 300 python bench.py --config dtu_eval_800x600_n5_d256 --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing > gpurun_out/${T}_cfg2_ms$ms.json 2> gpurun_out/${T}_cfg2_ms$ms.err || exit 1
  timeout -k 10 300 python bench.py --train --steps 3 > gpurun_out/${T}_train_ms$ms.json 2> gpurun_out/${T}_train_ms$ms.err || exit 1
done
unset AARMVS_CELL_MS
python tools/ab_summary.py gpurun_out/${T}_cfg1_ms0.json gpurun_out/${T}_cfg1_msauto.json gpurun_out/${T}_cfg2_ms0.json gpurun_out/${T}_cfg2_msauto.json
for f in gpurun_out/${T}_train_ms*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d.get('value'), d.get('unit'), d.get('ms_per_step'))"; done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.log
exit $rc
