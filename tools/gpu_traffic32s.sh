# split-fp32 PMC traffic of conv_layers.5 fwd / dgrad / wgrad at B = 1024 -> profiles JSONs (on the box)
cd $GRAFT_REPO_ROOT
for m in fwd dgrad wgrad; do
  bash tools/gpu_traffic32.sh c5 $m 1024 1 || exit $?
  python3 tools/traffic32.py gpurun_out/traffic32s_c5_${m}_1024 gpurun_out/traffic32s_neutron_c5_${m}_b1024.json c5 $m 1024 6 1 || exit $?
done
