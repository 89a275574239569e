#!/bin/bash
# cbw_feat blocks per CU (AARMVS_CBF_MINB 2 = the library, 3, 4: tools/ab/lib_cbf{3,4}.so) on the
# config-4 training step, A/B/C twice on one box, kernel averages from the timing pass.
set -o pipefail
T=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python bench.py --train --steps 3 > gpurun_out/${T}_m2_$r.json 2> gpurun_out/${T}_m2_$r.err || exit 1
  for m in 3 4; do
    AARMVS_LIB=$PWD/tools/ab/lib_cbf$m.so timeout -k 10 300 python bench.py --train --steps 3 > gpurun_out/${T}_m${m}_$r.json 2> gpurun_out/${T}_m${m}_$r.err || exit 1
  done
done
for f in gpurun_out/${T}_m*_*.json; do python -c "
import json; d=json.load(open('$f')); k=d['train_kernels']; k=k.get('kernels',k)
print('$f'.split('/')[-1], d['ms_per_step'], {n: round(v['avg_us'],1) for n, v in k.items() if n in ('cbw_feat','cbw_chain','head_wgrad')})"; done
