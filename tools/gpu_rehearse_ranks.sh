#!/bin/bash
# rehearsal of bench.py's multi-rank path on a one-GPU box: 2 and 4 ranks sharing the GPU
# (gloo), and the loud failure of --gpus 2 without the rehearsal switch
set -o pipefail
mkdir -p gpurun_out
python bench.py --gpus 2 --steps 1 > gpurun_out/ranks_refuse.log 2>&1; echo "unshared --gpus 2 rc=$? (expected 2)"
for n in 2 4; do
  AARMVS_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus $n --steps 2 --warmup 1 --no-cpu --no-fusion --no-e2e \
    --no-kernel-timing --planes 16 > gpurun_out/ranks_$n.log 2>&1 || { tail -20 gpurun_out/ranks_$n.log; exit 1; }
  grep '^{' gpurun_out/ranks_$n.log | cut -c1-420
done
AARMVS_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu --no-fusion --no-e2e --no-kernel-timing --planes 16 \
  > gpurun_out/ranks_torchrun.log 2>&1 || { tail -20 gpurun_out/ranks_torchrun.log; exit 1; }
grep '^{' gpurun_out/ranks_torchrun.log | cut -c1-420
