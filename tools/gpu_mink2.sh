# second A/B of ES_WGRAD_MINK: E=1 B=1024 (alternating) and E=4 B=512 at larger minimums
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
for m in 8 64 128 8 64 128; do
  ES_WGRAD_MINK=$m timeout -k 10 300 python bench.py --steps 200 --fp32-steps 0 --no-cpu-baseline --no-probe > $O/mk2_e1_m$m.json 2> $O/mk2_e1_m$m.err || exit $?
  echo "e1 b1024 mink=$m $(python -c "import json;d=json.load(open('$O/mk2_e1_m$m.json'));print(d['ms_per_step'])")"
done
for m in 64 128 256; do
  ES_WGRAD_MINK=$m timeout -k 10 300 python bench.py --batch 512 --experts 4 --steps 100 --warmup 120 --fp32-steps 0 --no-cpu-baseline --no-probe > $O/mk2_e4_m$m.json 2> $O/mk2_e4_m$m.err || exit $?
  echo "e4 mink=$m $(python -c "import json;d=json.load(open('$O/mk2_e4_m$m.json'));print(d['ms_per_step'])")"
done
for m in 8 128; do
  ES_WGRAD_MINK=$m timeout -k 10 300 python bench.py --batch 512 --steps 200 --fp32-steps 0 --no-cpu-baseline --no-probe > $O/mk2_b512_m$m.json 2> $O/mk2_b512_m$m.err || exit $?
  echo "e1 b512 mink=$m $(python -c "import json;d=json.load(open('$O/mk2_b512_m$m.json'));print(d['ms_per_step'])")"
done
