set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trprof -o run -- python3 $R/bench.py --train --steps 2 --warmup 1 --no-cpu --no-kernel-timing > $R/gpurun_out/trprof.log 2>&1
