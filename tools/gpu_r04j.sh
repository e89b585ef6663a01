# image-group size of the ring row order on the proton 4x4 convs (ES_RING_NG), alternating: 64 (default) / 16 / 8
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
for i in 1 2; do
  for g in 64 16 8; do
    ES_RING_NG=$g timeout -k 10 300 python bench.py --arch proton --batch 512 --steps 15 --other-steps 0 --no-cpu-baseline > $O/png${g}_$i.json 2> $O/png${g}_$i.err || exit $?
  done
done
