# norm NT A/B (fp32 bench shapes), proton fp32 B = 512 bench, proton conv_layers.1 / .5 PMC traffic (split-fp32)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
bash tools/gpu_norm_ab.sh n_base n_ld n_st n_ldst n_base n_ldst n_ld || exit $?
timeout -k 10 300 python bench.py --arch proton --batch 512 --steps 20 --other-steps 0 --no-cpu-baseline > $O/proton512_r04h.json 2> $O/proton512_r04h.err || exit $?
for L in p1 p5; do
  for m in fwd dgrad wgrad; do
    bash tools/gpu_traffic32.sh $L $m 1024 1 || exit $?
    python3 tools/traffic32.py $O/traffic32s_${L}_${m}_1024 $O/traffic32s_proton_${L}_${m}_b1024.json $L $m 1024 6 1 || exit $?
  done
done
# eager / data-parallel (RCCL world size 1) step cost against the graph replay
timeout -k 10 300 python bench.py --steps 20 --other-steps 0 --no-cpu-baseline --no-probe --graph off > $O/eager_r04h.json 2> $O/eager_r04h.err || exit $?
timeout -k 10 300 python bench.py --ddp --sync-bn --steps 20 --other-steps 0 --no-cpu-baseline --no-probe > $O/ddp1_r04h.json 2> $O/ddp1_r04h.err || exit $?
