set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06j
bash tools/gpu_r06i.sh || exit 1
bash tools/gpu_libab.sh ab_libs/libB_noslp.so 3 || exit 1
