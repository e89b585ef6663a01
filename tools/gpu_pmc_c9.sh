# FETCH / L2 hit counters of the c9 FWD conv launch, persistent kernel vs ring kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_c9
mkdir -p $O
export ES_MB_BATCH=1024
P="python3 $GRAFT_REPO_ROOT/tools/mb_one.py c9 fwd 1 5"
for v in 1 0; do
  export ES_PERSIST=$v
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$v -o run -- $P > $O/fetch_$v.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/hit_$v -o run -- $P > $O/hit_$v.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- $P > $O/kt_$v.log 2>&1 || exit 1
done
