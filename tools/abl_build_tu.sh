#!/bin/bash
# A/B builds of one translation unit: csrc/<tu>.hip recompiled with extra -D flags, linked with the
# regular objects into _abl/<name>/libexpertsim_hip.so (ES_LIB selects one at run time).
#   bash tools/abl_build_tu.sh <tu> name1 "-DFOO=1" name2 "-DFOO=2" ...
set -e
cd "$(dirname "$0")/.."
CS=generative-dnn-for-physics-simulations-cern_amd/csrc
TU=$1; shift
make -C $CS -j8 >/dev/null
names=()
while [ $# -ge 2 ]; do
  d=_abl/$1; mkdir -p $d; names+=($1)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $2 -c $CS/$TU.hip -o $d/$TU.o &
  shift 2
done
wait
for n in "${names[@]}"; do
  d=_abl/$n
  objs=$(ls $CS/build/*.o | grep -v "/$TU.o")
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libexpertsim_hip.so $objs $d/$TU.o
  rm -f $d/$TU.o
done
