#!/bin/bash
# Diagnostic builds of the ring kernel (ES_RING_EXP variants, see conv_mfma.hip) into
# tools/_exp/expN/: conv_mfma.hip recompiled, linked with the regular objects of csrc/build.
set -e
cd "$(dirname "$0")/.."
CS=generative-dnn-for-physics-simulations-cern_amd/csrc
make -C $CS -j8 >/dev/null
for n in "$@"; do
  d=tools/_exp/exp$n
  mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -DES_RING_EXP=$n -c $CS/conv_mfma.hip -o $d/conv_mfma.o &
done
wait
for n in "$@"; do
  d=tools/_exp/exp$n
  objs=$(ls $CS/build/*.o | grep -v conv_mfma.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libexpertsim_hip.so $objs $d/conv_mfma.o
  rm -f $d/conv_mfma.o
done
