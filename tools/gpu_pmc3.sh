# PMC passes over the three neutron G conv_layers.5 ops (tools/gpu_pmc.sh each)
set -o pipefail
cd $GRAFT_REPO_ROOT
for m in fwd dgrad wgrad; do bash tools/gpu_pmc.sh c5 $m 1 || exit 1; done
