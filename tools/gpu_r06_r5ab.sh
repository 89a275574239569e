#!/bin/bash
# Round 6 against round 5 on one box: the round-5 final tree (git worktree of 0e7fec6 at
# tools/ab/r05tree, its own library built there) as A and this tree as B -- the sweep digests
# (the round's kernel and schedule changes are bit-identical), then headline, config 2 and the
# training step, A/B/A/B.
set -o pipefail
mkdir -p gpurun_out
T=$1
A=$PWD/tools/ab/r05tree
(cd $A && timeout -k 10 200 python tools/sweep_digest.py) > gpurun_out/${T}_digest.txt 2>&1 || exit 1
timeout -k 10 200 python tools/sweep_digest.py >> gpurun_out/${T}_digest.txt 2>&1 || exit 1
cat gpurun_out/${T}_digest.txt
line() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], 'ms')" "$@"; }
for r in 1 2; do
  for side in A B; do
    dir=$PWD; [ $side = A ] && dir=$A
    (cd $dir && timeout -k 10 300 python bench.py --steps 3 --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing) > gpurun_out/${T}_h_${side}$r.json 2> gpurun_out/${T}_h_${side}$r.err || exit 1
    line gpurun_out/${T}_h_${side}$r.json headline_$side$r
    (cd $dir && timeout -k 10 300 python bench.py --config dtu_eval_800x600_n5_d256 --steps 3 --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing) > gpurun_out/${T}_c2_${side}$r.json 2> gpurun_out/${T}_c2_${side}$r.err || exit 1
    line gpurun_out/${T}_c2_${side}$r.json config2_$side$r
    (cd $dir && timeout -k 10 300 python bench.py --train --steps 4 --warmup 2 --no-cpu --no-kernel-timing) > gpurun_out/${T}_t_${side}$r.json 2> gpurun_out/${T}_t_${side}$r.err || exit 1
    line gpurun_out/${T}_t_${side}$r.json train_$side$r
  done
done 2>&1 | tee gpurun_out/${T}_summary.txt
