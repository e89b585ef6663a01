# fp32 ring variants of the generator convs at B=1024 (tools/mb_one.py, HIP-event timing)
cd $GRAFT_REPO_ROOT
export ES_MB_BATCH=1024 ES_MB_DTYPE=fp32
for L in c5 c0 c9; do for M in fwd dgrad wgrad; do
  for V in "" "ES_RING256=0" "ES_SP_MERGE=0" "ES_RING_NG=16"; do
    echo -n "$V: "; env $V timeout -k 10 60 python3 tools/mb_one.py $L $M 1 10 || exit $?
  done
done; done
