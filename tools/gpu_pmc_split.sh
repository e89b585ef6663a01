# PMC passes of the split-fp32 conv kernels: bash tools/gpu_pmc_split.sh <layer> <mode> [split 1|0]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
export ES_MB_DTYPE=fp32 ES_MB_SPLIT=${3:-1} ES_MB_BATCH=${ES_MB_BATCH:-1024}
O=$GRAFT_REPO_ROOT/gpurun_out/pmcs_$1_$2_${3:-1}
mkdir -p $O
P="python3 $GRAFT_REPO_ROOT/tools/mb_one.py $1 $2 1 3"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $P > $O/kt.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- $P > $O/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $O/p4 -o run -- $P > $O/p4.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAVES --output-format csv -d $O/p5 -o run -- $P > $O/p5.log 2>&1
