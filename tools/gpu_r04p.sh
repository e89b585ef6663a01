# thin Cout = 1 conv (conv_layers.13) with 1 / 2 / 4 channel chunks per lane: kernel tests per variant, then
# per-op timing at B = 1024 fp32 (split mode, deterministic wgrad), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
: > $O/k1.log
for c in 2 4; do
  ES_K1_CH=$c ES_K1_CH_WG=$c timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k "conv_fwd_dgrad_wgrad" --timeout 200 --timeout-method thread >> $O/k1.log 2>&1 || exit $?
done
export ES_MB_BATCH=1024 ES_MB_DTYPE=fp32 ES_MB_SPLIT=1
for i in 1 2; do
  for c in 1 2 4; do
    for m in fwd dgrad wgrad; do
      ES_K1_CH=$c ES_K1_CH_WG=$c timeout -k 10 120 python tools/mb_one.py c13 $m 1 20 2>/dev/null | sed "s/^/CH=$c /" >> $O/k1.log || exit $?
    done
  done
done
