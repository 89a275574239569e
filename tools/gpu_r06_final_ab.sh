#!/bin/bash
# Round-6 final evidence in one call: part A (GPU suite, smoke, rocprofv3 statistics of the
# headline, PMC ceiling and traffic passes) then part B (default bench line, configs)
set -o pipefail
bash tools/gpu_r06_final_a.sh $1 && bash tools/gpu_r06_final_b.sh $1
