# Run GPU steps in order; a step that exits with a test failure (1) lets the next run, anything
# else (fault, abort, timeout, signal) ends the script there.
#   bash tools/gpu_step.sh <outdir> "<name>:<timeout>:<command>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
worst=0
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; to=${rest%%:*}; cmd=${rest#*:}
  echo "[step] $name ($to s): $cmd"
  timeout -k 10 $to bash -c "$cmd" > $O/$name.log 2>&1
  rc=$?
  echo "[step] $name rc=$rc"; tail -3 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ $rc -gt $worst ] && worst=$rc
done
exit $worst
