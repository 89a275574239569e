#!/bin/bash
# Build diagnostic variants of libaarmvs.so with convlstm.hip compiled under -D flags into
# tools/ab/lib_NAME.so (A/B with AARMVS_LIB): bash tools/cell_variant.sh NAME "-DFLAG=..." ...
set -eu
cd "$(dirname "$0")/../aa-rmvsnet_amd/csrc"
make -s -j8 >/dev/null
mkdir -p ../../tools/ab/build
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -Xclang -target-feature -Xclang -packed-fp32-ops \
    $flags -c convlstm.hip -o ../../tools/ab/build/convlstm_$name.o
  objs=$(ls build/*.o | grep -v convlstm.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/ab/lib_$name.so \
    $objs ../../tools/ab/build/convlstm_$name.o
  echo "built tools/ab/lib_$name.so ($flags)"
done
