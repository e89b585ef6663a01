"""Evaluation on the HIP path against the reference's goldens and the oracle.

* es_channel_sums (csrc/eval.hip) vs the reference's sum_channels_parallel outputs and vs the
  oracle on ragged / strided / bf16 inputs; exact-partition property at a large size.
* the generator in eval mode (BatchNorm running statistics, no dropout) vs the reference's
  get_predictions_from_generator_results, with the reference's noise injected;
* calculate_joint_ws_across_experts with the reference's recorded torch.randn rows replayed.
Tolerances: sums of fp32 data <= 1e-6 relative (fp64 accumulation on both sides; the real-image
golden was summed in float32 by the reference: 1e-5); generated images <= 1e-4 relative to max|x|
(fp32 MFMA vs CPU); WS means <= 1e-4 relative, their std over repetitions
<= 1e-4 x the mean (absolute).
"""
import copy
import json
import os

import numpy as np
import pytest
import torch

from golden_utils import GOLDEN_DIR
from oracle import expertsim_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
ARCHES = ["neutron", "proton"]


def _golden(arch):
    z = np.load(os.path.join(GOLDEN_DIR, f"eval_{arch}.npz"), allow_pickle=False)
    return z, json.loads(str(z["meta"]))


def running_stats(n, expert):
    i = np.arange(n, dtype=np.float64)
    return ((0.1 * np.sin(0.37 * i + expert)).astype(np.float32),
            (0.75 + 0.25 * np.cos(0.11 * i + 2 * expert)).astype(np.float32))


def _generators(arch, seed):
    from expertsim.config import inject_shared, load_config
    from expertsim.models import build_model
    cfg = inject_shared(load_config(overrides=[f"model.architecture={arch}", "train.precision=fp32"]))
    torch.manual_seed(seed)
    g0 = build_model(f"{arch}.generator", cfg.model.generator, DEV)
    gens = [g0, copy.deepcopy(g0)]
    with torch.no_grad():
        for e, g in enumerate(gens):
            for m in g.modules():
                if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
                    mean, var = running_stats(m.num_features, e)
                    m.running_mean.copy_(torch.from_numpy(mean))
                    m.running_var.copy_(torch.from_numpy(var))
    return gens


@pytest.mark.parametrize("arch", ARCHES)
def test_channel_sums_golden(arch):
    from expertsim.train.utils import channel_sums, sum_channels_parallel
    z, _ = _golden(arch)
    real = torch.from_numpy(z["real_images"]).to(DEV)
    got = channel_sums(real, log_domain=True).cpu().numpy()
    np.testing.assert_allclose(got, z["ch_org"], rtol=1e-5, atol=1e-4)
    res = z["pred/res"].astype(np.float32)
    got2 = np.array(list(sum_channels_parallel(res)))          # reference API: host array in
    np.testing.assert_allclose(got2, z["pred/ch"], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("shape", [(0, 4, 4), (1, 1, 1), (5, 2, 3), (33, 7, 5), (257, 56, 30), (100, 44, 44),
                                   (9, 65, 67)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_channel_sums_vs_oracle(shape, dtype):
    from expertsim.train.utils import channel_sums
    g = torch.Generator().manual_seed(sum(shape))
    x = (torch.rand(shape, generator=g) * 3.0).to(dtype)
    xd = x.to(DEV)
    for log in (False, True):
        got = channel_sums(xd, log_domain=log).cpu().numpy()
        xf = x.float().numpy()
        ref = O.channel_sums(np.expm1(xf) if log else xf)
        np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-9)
    # strided view ([N,1,H,W] with a column stride of 2) and a [N,1,H,W] tensor
    if shape[0] > 0:
        wide = torch.zeros(shape[0], 1, shape[1], 2 * shape[2], dtype=dtype, device=DEV)
        wide[..., ::2] = xd[:, None]
        got = channel_sums(wide[..., ::2]).cpu().numpy()
        np.testing.assert_allclose(got, O.channel_sums(x.float().numpy()), rtol=1e-6, atol=1e-9)


def test_channel_sums_partition_large():
    """Full-size property: the five masks partition the image, so the channel sums add up to the
    photon sum (checksum of checksums) — 200k neutron-shaped images."""
    from expertsim.train.utils import channel_sums
    x = torch.rand(200_000, 44, 44, device=DEV)
    s = channel_sums(x)
    tot = x.double().sum(dim=(1, 2))
    assert torch.allclose(s.sum(1), tot, rtol=1e-9, atol=1e-9)
    assert bool((s >= 0).all())


@pytest.mark.parametrize("arch", ARCHES)
def test_eval_generator_matches_reference(arch):
    from expertsim.train.utils import get_predictions_from_generator_results
    z, meta = _golden(arch)
    gens = _generators(arch, meta["seed"])
    n = meta["n_pred"]
    shape = tuple(z["pred/raw"].shape[1:])
    res, raw = get_predictions_from_generator_results(3, n, 10, torch.device(DEV), torch.from_numpy(z["cond"][:n]),
                                                      gens[1], shape_images=shape,
                                                      input_noise=torch.from_numpy(z["pred/noise"]))
    ref = z["pred/raw"]
    assert np.abs(raw - ref).max() <= 1e-4 * max(np.abs(ref).max(), 1e-6)
    assert not gens[1].training      # left in eval mode, as the reference does (utils.py:195)


@pytest.mark.parametrize("arch", ARCHES)
def test_joint_ws_matches_reference(arch, monkeypatch):
    from expertsim.train import utils as U
    z, meta = _golden(arch)
    gens = _generators(arch, meta["seed"])
    rows = torch.from_numpy(z["ws/noise"])
    pos = [0]

    def replay(*size, device=None, **kw):
        n, d = size
        out = rows[pos[0]:pos[0] + n].to(device)
        assert out.shape == (n, d)
        pos[0] += n
        return out
    monkeypatch.setattr(U.torch, "randn", replay)
    assign, cond, ch_org = z["assign"], z["cond"], z["ch_org"]
    idx = [np.where(assign == e)[0] for e in range(2)]
    shape = tuple(z["real_images"].shape[1:])
    m, s, me, se = U.calculate_joint_ws_across_experts(
        meta["n_calc"], [z["real_images"][ix] for ix in idx], [torch.from_numpy(cond[ix]).to(DEV) for ix in idx],
        gens, ch_org, [ch_org[ix] for ix in idx], 10, torch.device(DEV), batch_size=1024, n_experts=2,
        shape_images=shape)
    monkeypatch.undo()
    assert pos[0] == rows.shape[0]
    scale = float(z["ws/mean"])
    np.testing.assert_allclose(m, scale, rtol=1e-4)
    np.testing.assert_allclose(me, z["ws/mean_exp"], rtol=1e-4)
    np.testing.assert_allclose(s, float(z["ws/std"]), rtol=0, atol=1e-4 * scale)
    np.testing.assert_allclose(se, z["ws/std_exp"], rtol=0, atol=1e-4 * scale)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_moe_evaluate_epoch(precision):
    """MoEWrapper.evaluate + loop.evaluate_epoch end to end (3 experts, synthetic test loader)."""
    from torch.utils.data import DataLoader, TensorDataset

    from expertsim.config import inject_shared, load_config
    from expertsim.train.loop import evaluate_epoch, setup_moe_system
    from expertsim.utils.synthetic import make_batch
    cfg = load_config(overrides=["model.architecture=neutron", "dataset.input_image_shape=[44,44]",
                                 "model.n_experts=3", f"train.precision={precision}",
                                 "model.router.diff_strength=1e-6"])
    torch.manual_seed(3)
    moe = setup_moe_system(cfg, torch.device(DEV))
    b = make_batch(96, "neutron", seed=11)
    x = torch.from_numpy(b["real_images"])
    ds = TensorDataset(x, x, torch.from_numpy(b["cond"]), torch.from_numpy(b["std"]),
                       torch.from_numpy(b["intensity"]), torch.from_numpy(b["true_positions"]))
    out = evaluate_epoch(moe, DataLoader(ds, batch_size=48), epoch=7, cfg=cfg, device=torch.device(DEV))
    keys = {"ws_mean", "ws_std", *[f"ws_mean_{i}" for i in range(3)], *[f"ws_std_{i}" for i in range(3)]}
    assert set(out) == keys
    assert all(np.isfinite(v) and v >= 0 for v in out.values())
    assert out["ws_mean"] > 0
