# HBM traffic + MFMA-busy of one neutron generator conv launch: separate rocprofv3 --pmc passes for
# FETCH_SIZE, WRITE_SIZE and SQ_VALU_MFMA_BUSY_CYCLES+GRBM_GUI_ACTIVE (MI355X_MICROARCH.md, HBM/rocprofv3
# section), plus a kernel-trace pass for the duration.
#   bash tools/gpu_traffic.sh <layer c5> <mode fwd> <batch 512>
# Output under gpurun_out/traffic_<layer>_<mode>_<batch>/ (tools/traffic_json.py turns it into
# profiles/traffic_neutron_<layer>_<mode>_b<batch>.json, which bench.py reports as roofline.traffic).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
L=${1:-c5}; M=${2:-fwd}; NB=${3:-512}
O=$GRAFT_REPO_ROOT/gpurun_out/traffic_${L}_${M}_${NB}
mkdir -p $O
export ES_MB_BATCH=$NB
P="python3 $GRAFT_REPO_ROOT/tools/mb_one.py $L $M 1 5"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $P > $O/kt.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $P > $O/fetch.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $P > $O/write.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/mfma -o run -- $P > $O/mfma.log 2>&1
