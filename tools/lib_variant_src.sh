#!/bin/bash
# Build the in-tree sources as they stand into tools/ab/lib_NAME.so (the in-tree library is left
# as it was): bash tools/lib_variant_src.sh NAME
set -eu
cd "$(dirname "$0")/../aa-rmvsnet_amd/csrc"
mkdir -p ../../tools/ab/build_$1
for f in api warp_cost convlstm fusion group_norm lstm_train bptt evidential deform; do
  extra=""
  case $f in warp_cost|fusion|deform) extra="-ffp-contract=off";; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -Xclang -target-feature -Xclang -packed-fp32-ops $extra -c $f.hip -o ../../tools/ab/build_$1/$f.o 2>/dev/null &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/ab/lib_$1.so ../../tools/ab/build_$1/*.o
echo "built tools/ab/lib_$1.so"
