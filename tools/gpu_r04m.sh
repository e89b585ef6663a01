# vector deterministic WGRAD reduce (wgrad_reduce4_kernel): bitwise against the scalar kernel, then A/B on
# the bench (E = 1 B = 1024 and E = 4 B = 512), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
ES_WGRAD_REDUCE4=0 timeout -k 10 200 python tools/wr4_check.py $O/wr4_0.npz > $O/wr4.log 2>&1 || exit $?
ES_WGRAD_REDUCE4=1 timeout -k 10 200 python tools/wr4_check.py $O/wr4_1.npz >> $O/wr4.log 2>&1 || exit $?
python tools/wr4_check.py --compare $O/wr4_0.npz $O/wr4_1.npz >> $O/wr4.log 2>&1 || exit $?
for i in 1 2; do
  for v in 0 1; do
    ES_WGRAD_REDUCE4=$v timeout -k 10 300 python bench.py --steps 30 --other-steps 0 --no-cpu-baseline --no-probe > $O/wr4b${v}_$i.json 2> $O/wr4b${v}_$i.err || exit $?
  done
done
for v in 0 1; do
  ES_WGRAD_REDUCE4=$v timeout -k 10 300 python bench.py --experts 4 --batch 512 --steps 20 --other-steps 0 --no-cpu-baseline --no-probe > $O/wr4e4${v}.json 2> $O/wr4e4${v}.err || exit $?
done
