# SPB4 A/B (bitwise + timing) then PMC passes of the split c5 fwd / dgrad on the default (4-wave) kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 180 python tools/mb_spb4.py 1024 5 > gpurun_out/mb_spb4_r04b.log 2>&1 || exit $?
bash tools/gpu_pmc_split.sh c5 fwd 1 && bash tools/gpu_pmc_split.sh c5 dgrad 1
