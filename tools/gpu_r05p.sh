set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_deform.py tests/test_gpu_models.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05p_tests.log 2>&1 && \
timeout -k 10 400 python bench.py --train --steps 3 --warmup 1 --no-cpu > gpurun_out/r05p_train.json 2> gpurun_out/r05p_train.err
