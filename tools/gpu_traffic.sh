# HBM traffic of the roofline kernel (neutron G conv_layers.5 forward): separate rocprofv3 --pmc
# passes for FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md, HBM/rocprofv3 section), plus a
# kernel-trace pass for its duration.  Output under gpurun_out/traffic/ (tools/traffic_json.py
# turns it into profiles/<tag>_c5_fwd_traffic.json, which bench.py reports as roofline.traffic).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/traffic
mkdir -p $O
P="python3 $GRAFT_REPO_ROOT/tools/mb_one.py c5 fwd 1 5"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $P > $O/kt.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $P > $O/fetch.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $P > $O/write.log 2>&1
