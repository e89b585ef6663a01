# split-fp32 PMC traffic of the conv_layers.5 / .9 WGRAD at B = 1024 -> profiles JSONs (on the box)
cd $GRAFT_REPO_ROOT
for l in c5 c9; do
  bash tools/gpu_traffic32.sh $l wgrad 1024 1 || exit $?
  python3 tools/traffic32.py gpurun_out/traffic32s_${l}_wgrad_1024 gpurun_out/traffic32s_neutron_${l}_wgrad_b1024.json $l wgrad 1024 6 1 || exit $?
done
