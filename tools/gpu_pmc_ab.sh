# PMC passes over an alternating A/B of one split-fp32 op (both arms' kernels in each pass):
#   bash tools/gpu_pmc_ab.sh <tag> <layer> <mode> <switch> [batch]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/mb_ab.py $2 $3 $4 ${5:-1024} 1 3 ${6:-0,1}"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $P > $O/kt.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- $P > $O/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $O/p2 -o run -- $P > $O/p2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAVES SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_COEXEC_CYCLES --output-format csv -d $O/p3 -o run -- $P > $O/p3.log 2>&1
