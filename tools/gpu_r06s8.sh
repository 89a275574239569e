#!/bin/bash
# Round-6 training backward: head_wgrad / gnb_partial A/B on the config-4 training step
# (tools/ab/lib_base.so = the previous commit vs the in-tree library, A/B/A/B, one box, with the
# kernel-timing pass), then the GPU suite.
set -o pipefail
T=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  AARMVS_LIB=$PWD/tools/ab/lib_base.so timeout -k 10 300 python bench.py --train --steps 3 > gpurun_out/${T}_A_$r.json 2> gpurun_out/${T}_A_$r.err || exit 1
  timeout -k 10 300 python bench.py --train --steps 3 > gpurun_out/${T}_B_$r.json 2> gpurun_out/${T}_B_$r.err || exit 1
done
for f in gpurun_out/${T}_[AB]_*.json; do python -c "
import json; d=json.load(open('$f')); k=(d.get('train_kernels') or {}).get('kernels', d.get('train_kernels') or {})
print('$f'.split('/')[-1], d['ms_per_step'], {n: round(v['avg_us'],1) for n, v in k.items() if n in ('head_wgrad','gnb_partial','deconv_bwd','wgrad0','cbw_feat')})"; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.log
exit $rc
