# PMC passes of the fused discriminator front (d_front2.hip) at B = 1024 (tools/mb_dfront2.py): kernel
# trace, FETCH_SIZE, WRITE_SIZE, MFMA / VALU busy, in separate rocprofv3 runs
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_dfront2
mkdir -p $O
P="python3 $GRAFT_REPO_ROOT/tools/mb_dfront2.py 1024"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $P > $O/kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $P > $O/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $P > $O/write.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/busy -o run -- $P > $O/busy.log 2>&1
