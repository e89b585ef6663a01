#!/bin/bash
# Runs several short bench.py lines on one box, one JSON per line into gpurun_out/<tag>_<i>.json.
# usage: tools/gpu_bench_set.sh TAG "args1" "args2" ...   (each args string is passed to bench.py)
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
i=0
for a in "$@"; do
  echo "[$tag $i] bench.py $a"
  timeout -k 10 300 python bench.py $a > gpurun_out/${tag}_$i.json 2> gpurun_out/${tag}_$i.log || { echo "FAILED rc=$? ($a)"; tail -20 gpurun_out/${tag}_$i.log; exit 1; }
  cat gpurun_out/${tag}_$i.json
  i=$((i+1))
done
