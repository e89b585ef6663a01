# A/B of library builds under _abl/<name>/ (tools/abl_build_tu.sh) on the default bench, alternating:
#   bash tools/gpu_libab.sh base_name other1 other2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
: > $O/libab.log
run() {
  ES_LIB=$PWD/_abl/$1/libexpertsim_hip.so timeout -k 10 300 python bench.py --steps 30 --other-steps 0 --no-cpu-baseline ${BENCH_ARGS:-} > $O/libab.json 2> $O/libab.err || return $?
  python3 -c "import json; d=json.load(open('$O/libab.json')); r=d['roofline']; print('$1', d['ms_per_step'], {k: v['avg_ms'] for k, v in r['all_probed'].items()})" >> $O/libab.log
}
base=$1; shift
for i in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    run $base || exit $?
    run $v || exit $?
  done
done
run $base
