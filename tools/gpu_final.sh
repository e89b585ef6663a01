# round-end state: GPU suite, smoke(), the default bench line (as the driver runs it), a
# kernel-trace profile of the bench, and PMC traffic passes of conv_layers.9 and .5
#   bash tools/gpu_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-final}
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread > $O/t_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/t_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --fp32-steps 0 --no-cpu-baseline --graph off > $O/prof_$TAG.log 2>&1 && \
bash $GRAFT_REPO_ROOT/tools/gpu_traffic.sh c5 fwd 1024 && \
bash $GRAFT_REPO_ROOT/tools/gpu_traffic.sh c9 fwd 1024 && \
bash $GRAFT_REPO_ROOT/tools/gpu_traffic.sh c9 dgrad 1024 && \
bash $GRAFT_REPO_ROOT/tools/gpu_traffic.sh c9 wgrad 1024
