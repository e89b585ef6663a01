# PMC of the forward norm kernels in tools/mb_norm.py (instruction mix / instruction-fetch waits)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_norm
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU --kernel-include-regex bn_fwd_fast --output-format csv -d $O/p1 -o run -- python3 $GRAFT_REPO_ROOT/tools/mb_norm.py > $O/p1.log 2>&1
