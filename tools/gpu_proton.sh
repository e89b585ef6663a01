# proton 56x30 at reference precision (fp32 split) B = 512 / 1024, and the default neutron line: <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python bench.py --arch proton --batch 1024 --steps 20 --other-steps 0 --no-cpu-baseline > $O/proton1024_$1.json 2> $O/proton1024_$1.err && \
timeout -k 10 300 python bench.py --arch proton --batch 512 --steps 20 --other-steps 0 --no-cpu-baseline > $O/proton512_$1.json 2> $O/proton512_$1.err && \
timeout -k 10 300 python bench.py --steps 30 --other-steps 0 --no-cpu-baseline > $O/neutron_$1.json 2> $O/neutron_$1.err
