"""bench.py end to end (the driver's contract): one JSON line on stdout with the metric, the whole-job
value, the roofline object of the probed generator conv and the other-precision leg; for E > 1
(dynamic rows) the roofline sums each c5 op type over the experts' eager ops.  Small batches and few
steps: this checks the control flow and the line's shape, not the numbers."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", *args],
                       cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_line_e1():
    d = _bench("--batch", "64", "--steps", "3", "--warmup", "2", "--other-steps", "2")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 2 and d["dtype"] == "fp32"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert abs(d["value"] - 64 * 1000.0 / d["ms_per_step"]) <= 0.01 * d["value"]
    roof = d["roofline"]
    assert roof["bound"] == "mfma" and roof["unit"] == "TFLOP/s" and 0 < roof["frac"] < 1
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    assert d["perf_bf16"]["dtype"] == "bf16" and d["perf_bf16"]["value"] > 0


def test_bench_line_multi_expert():
    d = _bench("--experts", "4", "--batch", "128", "--steps", "3", "--warmup", "2", "--other-steps", "0")
    assert d["config"]["n_experts"] == 4 and d["value"] > 0
    # the E > 1 roofline: every expert's c5 ops probed in eager steps, work scaled by the routed shares
    r = d["roofline"]
    assert r["kernel"].startswith("G*.c5.") and "dynamic rows" in r["note"] and 0 < r["frac"] < 1, r
    assert set(r["all_probed"]) == {"G*.c5.fwd", "G*.c5.dgrad", "G*.c5.wgrad"}
