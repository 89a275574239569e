#!/bin/bash
# Round-6 step i: training tests (head weight gradient rewrite), the default bench line without
# the CPU / fusion / e2e legs (headline + config-4 training step with kernel table), then the
# omega-bias signed-error diagnostic over seeds.
set -o pipefail
mkdir -p gpurun_out
T=$1
timeout -k 10 500 python -u -m pytest tests/test_gpu_bptt.py tests/test_gpu_training.py tests/test_gpu_train_fixtures.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -20 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 500 python -u bench.py --no-cpu --no-fusion --no-e2e --steps 2 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
python - <<PY
import json
d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().split('\n')[-1])
print('headline', d['value']/1e9, d['ms_per_step'])
t=d['train']; print('train', t['s_per_step'], t['ms_per_plane'], t.get('s_per_step_one_stream'))
k=t['kernels']; print({n: k[n]['avg_us'] for n in ('head_wgrad','cbw_feat','wgrad0','dgrad0','lstm_cell0') if n in k})
PY
timeout -k 10 900 python -u tests/diag_omega_bias_seeds.py 6 1 3 32 48 6 > gpurun_out/${T}_bias_a.txt 2>&1
tail -8 gpurun_out/${T}_bias_a.txt
