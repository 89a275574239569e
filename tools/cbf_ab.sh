#!/bin/bash
# Build diagnostic variants of libaarmvs.so (warp_cost.hip with -D flags) into tools/ab/ for
# A/B timing with AARMVS_LIB (tools/cbf_probe.py).  usage: bash tools/cbf_ab.sh NAME "-DFLAG=..." ...
set -eu
cd "$(dirname "$0")/../aa-rmvsnet_amd/csrc"
make -s -j8 >/dev/null
mkdir -p ../../tools/ab/build
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -ffp-contract=off -Xclang -target-feature -Xclang -packed-fp32-ops \
    $flags -c warp_cost.hip -o ../../tools/ab/build/warp_cost_$name.o
  objs=$(ls build/*.o | grep -v warp_cost.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/ab/lib_$name.so \
    $objs ../../tools/ab/build/warp_cost_$name.o
  echo "built tools/ab/lib_$name.so ($flags)"
done
