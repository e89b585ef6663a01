"""Checkpoint / resume and EMA on the HIP path.

* es_ema_update is bit-exact against the reference's EMAHelper.update arithmetic
  (expertsim/train/loop.py:398-399: ``decay*shadow + (1-decay)*param`` in fp32 torch on the CPU);
* a checkpoint restores bit-exactly every piece of state (weights, BatchNorm / spectral-norm
  buffers, Adam moments and step counts, EMA shadow, device RNG keys) into a differently
  initialised model, and the resumed run continues the saved one: the next steps' metrics agree
  to 1e-3 relative and parameters to 2*lr per step (not bitwise: the fp32 weight-gradient and
  norm-statistics reductions use float atomics, so two runs of one step differ in the last ulp);
* every file loads with weights_only=True.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("n,off", [(1, 0), (7, 0), (4096, 0), (100003, 1), (64 * 1024 + 5, 3)])
def test_ema_update_matches_reference_arithmetic(n, off):
    from expertsim import hip
    g = torch.Generator().manual_seed(n)
    s = torch.randn(n + off, generator=g)
    p = torch.randn(n + off, generator=g) * 3
    decay = 0.99
    want = decay * s[off:] + (1.0 - decay) * p[off:]          # the reference's EMAHelper.update
    sd, pd = s.to(DEV), p.to(DEV)
    hip.call("es_ema_update", hip.ptr(sd[off:]), hip.ptr(pd[off:]), n, decay, 1.0 - decay, hip.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(sd[off:].cpu(), want)
    assert torch.equal(sd[:off].cpu(), s[:off])


def _setup(seed=1234, arch="neutron", E=1):
    from expertsim.config import inject_shared, load_config
    from expertsim.train.loop import setup_moe_system
    from expertsim.train.training_setup import setup_optimizers
    cfg = inject_shared(load_config(overrides=[f"model.architecture={arch}", f"model.n_experts={E}",
                                               "train.precision=fp32", f"train.rng_seed={seed}",
                                               "dataset.input_image_shape=" + ("[44,44]" if arch == "neutron" else "[56,30]")]))
    torch.manual_seed(seed)
    moe = setup_moe_system(cfg, torch.device(DEV))
    return moe, setup_optimizers(moe, cfg), cfg


def _batch(arch, B, seed):
    from expertsim.utils.synthetic import make_batch
    b = make_batch(B, arch, seed=seed)
    return [torch.from_numpy(b[k]).to(DEV) for k in ("cond", "real_images", "true_positions", "std", "intensity")]


def _step(moe, opts, batch, epoch=0):
    og, od, oa, orr = opts
    cond, img, pos, std, inten = batch
    m = moe.train_step(epoch, cond, img.unsqueeze(1), pos, std, inten, oa, og, od, orr, None, DEV)
    return {k: float(v) for k, v in m.items() if torch.is_tensor(v) and v.numel() == 1}


@pytest.mark.parametrize("arch,E", [("neutron", 1), ("proton", 2)])
def test_resume_restores_state(tmp_path, arch, E):
    from expertsim.train.ema import EMAHelper
    from expertsim.train.training_utils import load_checkpoint, save_checkpoint
    B = 8 * E
    batches = [_batch(arch, B, s) for s in range(4)]
    moe, opts, _ = _setup(arch=arch, E=E)
    ema = EMAHelper(moe, 0.99)
    for b in batches[:2]:
        _step(moe, opts, b)
        ema.update(moe, range(E))
    save_checkpoint(str(tmp_path), 1, moe, *opts, ema_helper=ema)
    saved = {k: v.detach().cpu().clone() for k, v in moe.state_dict().items()}
    saved_opt = [o.state_dict() for group in opts[:3] for o in group] + [opts[3].state_dict()]
    cont = [_step(moe, opts, b) for b in batches[2:]]
    params_a = [p.detach().cpu().clone() for p in moe.parameters()]

    moe2, opts2, _ = _setup(seed=99, arch=arch, E=E)          # different init: everything must be loaded
    ema2 = EMAHelper(moe2, 0.5)
    st = load_checkpoint(str(tmp_path), 1, moe2, *opts2, ema_helper=ema2, device=DEV)
    assert st["step_count"] == 2 and ema2.decay == 0.99
    for i in range(E):                                        # the EMA was not advanced after the save
        for k in ema.shadow[i]:
            assert torch.equal(ema.shadow[i][k].cpu(), ema2.shadow[i][k].cpu()), k
    for k, v in moe2.state_dict().items():
        assert torch.equal(saved[k], v.detach().cpu()), k
    loaded_opt = [o.state_dict() for group in opts2[:3] for o in group] + [opts2[3].state_dict()]
    for a, b in zip(saved_opt, loaded_opt):
        assert a["step"] == b["step"] and torch.equal(a["exp_avg"], b["exp_avg"])
        assert torch.equal(a["exp_avg_sq"], b["exp_avg_sq"])
    resumed = [_step(moe2, opts2, b) for b in batches[2:]]
    for a, r in zip(cont, resumed):
        for k in a:
            assert abs(a[k] - r[k]) <= 1e-3 * max(abs(a[k]), 1e-3) or (np.isnan(a[k]) and np.isnan(r[k])), \
                (k, a[k], r[k])
    lr = max(o.param_groups[0]["lr"] for group in opts2[:3] for o in group)
    for pa, pb in zip(params_a, moe2.parameters()):
        assert float((pa - pb.detach().cpu()).abs().max()) <= 2 * lr * len(batches[2:]) + 1e-7
    for f in os.listdir(tmp_path):
        torch.load(os.path.join(tmp_path, f), map_location="cpu", weights_only=True)


def test_ema_apply_and_restore():
    from expertsim.train.ema import EMAHelper
    moe, opts, _ = _setup()
    ema = EMAHelper(moe, 0.9)
    p0 = moe.generators[0].flat_params.clone()
    _step(moe, opts, _batch("neutron", 8, 0))
    p1 = moe.generators[0].flat_params.clone()
    assert not torch.equal(p0, p1)
    ema.update(moe, [0])
    want = 0.9 * p0.cpu() + (1.0 - 0.9) * p1.cpu()
    flat_shadow = torch.cat([v.reshape(-1) for v in ema.shadow[0].values()]).cpu()
    assert torch.equal(flat_shadow, want)
    ema.apply_shadow(moe)
    assert torch.equal(moe.generators[0].flat_params.cpu(), want)
    ema.restore(moe)
    assert torch.equal(moe.generators[0].flat_params, p1)
