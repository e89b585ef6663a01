# fp32 parity-mode HBM traffic + MFMA busy of one neutron generator conv op (separate rocprofv3
# passes, MI355X_MICROARCH.md HBM / rocprofv3 section):  bash tools/gpu_traffic32.sh <c5> <fwd> <1024> [split 0|1]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
L=${1:-c5}; M=${2:-fwd}; NB=${3:-1024}; SPL=${4:-0}
O=$GRAFT_REPO_ROOT/gpurun_out/traffic32$([ "$SPL" = 1 ] && echo s)_${L}_${M}_${NB}
mkdir -p $O
export ES_MB_BATCH=$NB ES_MB_DTYPE=fp32 ES_MB_SPLIT=$SPL
P="python3 $GRAFT_REPO_ROOT/tools/mb_one.py $L $M 1 5"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $P > $O/kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $P > $O/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $P > $O/write.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/mfma -o run -- $P > $O/mfma.log 2>&1
