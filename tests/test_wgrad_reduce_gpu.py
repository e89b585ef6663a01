"""The vectorised deterministic weight-gradient reduce (conv_mfma.hip wgrad_reduce4_kernel, 16-byte
partial loads) against the scalar kernel it replaces (ES_WGRAD_REDUCE4=0): per output the same
summation order, so the weight and bias gradients of the bench's conv shapes (neutron conv_layers.0 /
.5 / .9, proton conv_layers.1, the discriminator's 32 -> 16 and the aux regressor's 1 -> 32 convs) must
be bitwise equal.  The switch is read when the library loads, so each side runs in its own process
(tools/wr4_check.py)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(300)
def test_wgrad_reduce4_bitwise_equal_scalar(tmp_path):
    outs = []
    for v in ("0", "1"):
        out = tmp_path / f"wr4_{v}.npz"
        env = dict(os.environ, ES_WGRAD_REDUCE4=v)
        r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "wr4_check.py"), str(out)], env=env,
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(np.load(out))
    a, b = outs
    assert set(a.files) == set(b.files) and len(a.files) == 12
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    assert not bad, bad
    assert all(np.abs(a[k]).max() > 0 for k in a.files if not k.endswith(".bias"))
