set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06h
for v in 11 12 13 14; do timeout -k 10 120 python -u tools/mb_ab.py c5 wgrad es_conv_set_wgrad_ws 1024 2 10 1,$v | tail -1 || exit 1; done
