set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/microbench/cell_bench > gpurun_out/cell_bench.log 2>&1; rc=$?
cat gpurun_out/cell_bench.log | grep -v amdgpu.ids
exit $rc
