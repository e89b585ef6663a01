# thin conv grid caps (ES_K1_GRID for fwd / dgrad, ES_THIN_WGRID for wgrad) at B = 1024 fp32, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
: > $O/k1g.log
export ES_MB_BATCH=1024 ES_MB_DTYPE=fp32 ES_MB_SPLIT=1
for i in 1 2; do
  for g in 2048 0 4096 1024; do
    for m in fwd dgrad; do
      ES_K1_GRID=$g timeout -k 10 120 python tools/mb_one.py c13 $m 1 20 2>/dev/null | sed "s/^/K1_GRID=$g /" >> $O/k1g.log || exit $?
    done
  done
  for g in 1024 2048 512 4096; do
    ES_THIN_WGRID=$g timeout -k 10 120 python tools/mb_one.py c13 wgrad 1 20 2>/dev/null | sed "s/^/WGRID=$g /" >> $O/k1g.log || exit $?
  done
done
