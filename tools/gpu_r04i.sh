# A/B of the wide-linear pixel view (ES_LIN_PIX) on one box, alternating; proton fp32 B = 512 bench;
# proton conv_layers.1 / .5 PMC traffic (split-fp32, B = 1024)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
for i in 1 2; do
  for v in 0 1; do
    ES_LIN_PIX=$v timeout -k 10 300 python bench.py --steps 30 --other-steps 0 --no-cpu-baseline --no-probe > $O/linpix${v}_$i.json 2> $O/linpix${v}_$i.err || exit $?
  done
done
timeout -k 10 300 python bench.py --arch proton --batch 512 --steps 20 --other-steps 0 --no-cpu-baseline > $O/proton512_r04i.json 2> $O/proton512_r04i.err || exit $?
for L in p1 p5; do
  for m in fwd dgrad wgrad; do
    bash tools/gpu_traffic32.sh $L $m 1024 1 || exit $?
    python3 tools/traffic32.py $O/traffic32s_${L}_${m}_1024 $O/traffic32s_proton_${L}_${m}_b1024.json $L $m 1024 6 1 || exit $?
  done
done
