set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_fusion.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r02_eval_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r02_eval_tests.log
exit $rc
