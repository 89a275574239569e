#!/bin/bash
# omega_mfma items-per-block experiment: digests under several IPB, then headline A/Bs
set -o pipefail
mkdir -p gpurun_out
for v in 1 3 8; do
  AARMVS_OMEGA_IPB=$v timeout -k 10 200 python tools/sweep_digest.py >> gpurun_out/ipb_digest.txt 2>&1 || exit 1
done
bash tools/gpu_env_ab.sh ipb AARMVS_OMEGA_IPB 2 1 || exit 1
bash tools/gpu_env_ab.sh ipb4 AARMVS_OMEGA_IPB 4 8
