set -e
for p in 1 0; do
  echo "P256=$p"; ES_P256=$p timeout -k 10 120 python tools/ring_exp.py 1024
done
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv" 2>&1 | grep -v Warn | grep "^E \|^>\|passed\|failed" | head -30
