"""bf16 ring convolutions over image chunks.

The ring kernels address their gathered operand with 32-bit buffer offsets (out-of-range marker at
2^31), so operands of >= 1 GiB launch as image chunks (es_conv_ring_launch): a capacity-2048 expert's
conv_layers.5 output gradient is 1.1 GB in bf16 (BASELINE configs[3], E = 4, B = 2048 on one GPU),
which before the chunks fell back to the generic GEMM kernels (c5 WGRAD 5.3 ms instead of ~1.3).
Forced small chunks (es_conv_set_f32_chunk, the same knob as the fp32 ring) must give the FWD /
DGRAD of the whole-batch launch bit for bit (each output element's K order does not depend on the
row tiling) and its WGRAD up to the order of the float atomics; against torch fp64 within the bf16
tolerance of tests/test_kernels_gpu.py.

Reference: upsample + conv2d of neutron/generator.py:23-35 (torch CPU fp64).
"""
import pytest
import torch

from test_f32_ring_gpu import _ref
from test_kernels_gpu import DEV, _hip, from_act, rel, to_act

pytestmark = pytest.mark.gpu

CASES = [
    (130, 256, 24, 24, 128, 3, 1, 0, 2),   # neutron G conv_layers.5 (sub-pixel), ragged last chunk
    (70, 128, 46, 46, 64, 2, 1, 0, None),  # neutron G conv_layers.9
]


def _run(case, x, w, b, gy):
    from expertsim.layers import ConvOp, Upsample
    N, Cin, H, W, Cout, k, st, pad, up = case
    upsample = Upsample((H, W), scale=(up, up)) if up else None
    op = ConvOp(torch.nn.Parameter(w.to(DEV)), torch.nn.Parameter(b.to(DEV)), stride=st, pad=pad, upsample=upsample)
    xa = to_act(x, torch.bfloat16)
    ya = op.fwd(xa, out_dtype=torch.bfloat16)
    gya = to_act(gy, torch.bfloat16)
    dxa = op.dgrad(gya, xa, dx_dtype=torch.bfloat16)
    dw = torch.zeros_like(op.weight)
    op.wgrad(gya, xa, dw, None, beta=1.0)
    torch.cuda.synchronize()
    return from_act(ya).float(), from_act(dxa).float(), dw.cpu()


@pytest.fixture
def perf_mode():
    from expertsim import layers
    old = layers.deterministic()
    layers.set_deterministic(False)
    yield
    layers.set_deterministic(old)


@pytest.mark.parametrize("case", CASES)
def test_bf16_ring_image_chunks(case, perf_mode):
    hip = _hip()
    x, w, b, gy, y, gx, gw, gb = _ref(case, seed=7)
    full = _run(case, x, w, b, gy)
    launches = hip.lib().es_conv_launch_count()
    old = hip.lib().es_conv_set_f32_chunk(64)
    try:
        part = _run(case, x, w, b, gy)
    finally:
        hip.lib().es_conv_set_f32_chunk(old)
    # the chunked pass launched ring kernels per chunk (not the generic fallback)
    assert hip.lib().es_conv_launch_count() - launches >= 3 * ((case[0] + 63) // 64) - 1
    assert torch.equal(full[0], part[0])
    assert torch.equal(full[1], part[1])
    assert rel(part[2].double(), gw) < 2e-2
    assert rel(part[2], full[2]) < 1e-3
    assert rel(part[0].double(), y) < 2e-2
    assert rel(part[1].double(), gx) < 2e-2
