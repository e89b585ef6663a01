# round-4 check: SPB4 A/B (bitwise + timing), GPU suite + smoke + default bench, then one profiled bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 180 python tools/mb_spb4.py 1024 5 > gpurun_out/mb_spb4_r04a.log 2>&1 || exit $?
bash tools/gpu_verify.sh r04a || exit $?
bash tools/gpu_prof_bench.sh r04a
