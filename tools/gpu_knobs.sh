# A/B of tuning switches on the default bench (B = 1024 fp32), each alternated with the default on one box:
#   bash tools/gpu_knobs.sh "ES_SPB_NOSHORTK=1" "ES_SPL_PRIO=0" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
: > $O/knobs.log
run() {  # <label> <env...>
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --other-steps 0 --no-cpu-baseline --no-probe > $O/knob.json 2> $O/knob.err || return $?
  python3 -c "import json; d=json.load(open('$O/knob.json')); print('$lab', d['ms_per_step'])" >> $O/knobs.log
}
for k in "$@"; do
  run default ES_DUMMY=0 || exit $?
  run "$k" $k || exit $?
done
run default ES_DUMMY=0 || exit $?
