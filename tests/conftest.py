import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "generative-dnn-for-physics-simulations-cern_amd")
for p in (PKG_DIR, REPO, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    # the tests pin the default build and kernel paths: no ES_* environment override (ES_LIB would load
    # another build of the library)
    stray = sorted(k for k in os.environ if k.startswith("ES_"))
    if stray:
        raise pytest.UsageError(f"refusing to run with experimental switches set: {', '.join(stray)}")
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — run on the GPU box")
    config.addinivalue_line("markers", "slow: long-running CPU test")
