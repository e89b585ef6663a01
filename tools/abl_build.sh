#!/bin/bash
# A/B builds of the 4-wave split-fp32 kernels: conv_spb4.hip recompiled with extra -D flags, linked with
# the regular objects into _abl/<name>/libexpertsim_hip.so (ES_LIB selects one at run time).
#   bash tools/abl_build.sh name1 "-DFOO=1 -DBAR=2" name2 "-DFOO=2" ...
set -e
cd "$(dirname "$0")/.."
CS=generative-dnn-for-physics-simulations-cern_amd/csrc
make -C $CS -j8 >/dev/null
names=()
while [ $# -ge 2 ]; do
  d=_abl/$1; mkdir -p $d; names+=($1)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form \
    -fno-slp-vectorize $2 -c $CS/conv_spb4.hip -o $d/conv_spb4.o &
  shift 2
done
wait
for n in "${names[@]}"; do
  d=_abl/$n
  objs=$(ls $CS/build/*.o | grep -v conv_spb4.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libexpertsim_hip.so $objs $d/conv_spb4.o
  rm -f $d/conv_spb4.o
done
