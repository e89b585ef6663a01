# round-4 PMC traffic of the final kernels: conv_layers.5 fwd / dgrad / wgrad and conv_layers.9 fwd / dgrad /
# wgrad at B = 1024, split-fp32 (profiles/traffic32s_neutron_*_b1024.json)
cd $GRAFT_REPO_ROOT
for L in c5 c9; do
  for m in fwd dgrad wgrad; do
    bash tools/gpu_traffic32.sh $L $m 1024 1 || exit $?
    python3 tools/traffic32.py gpurun_out/traffic32s_${L}_${m}_1024 gpurun_out/traffic32s_neutron_${L}_${m}_b1024.json $L $m 1024 6 1 || exit $?
  done
done
