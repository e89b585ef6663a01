# round-4 check: GPU suite + smoke + default bench, then one profiled bench of the same tree: <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_verify.sh $1 || exit $?
bash tools/gpu_prof_bench.sh $1
