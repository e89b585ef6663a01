"""Checkpoint parity against the reference's module naming and forward (SURVEY.md
§8(f) row 3).

The reference saves whole modules (``save_models_and_architectures``, training_utils.py:316-381) and
its intended loader (``load_checkpoint_weights``, training_setup.py:70-214) restores them by their
``state_dict`` keys.  The build saves ``state_dict``s under the same file names.  Here:

* the key set and tensor shapes of every saved generator / discriminator / aux-regressor / router
  state_dict equal the reference's own ``state_dict`` keys, as the golden capture recorded them
  from the reference modules (tests/golden/*.npz ``init/<G|D|A|R>/<key>``);
* a checkpoint written after two HIP training steps is loaded (``torch.load(weights_only=True)``)
  straight into the oracle — the CPU restatement that takes the reference's parameter names and is
  bit-exact to the reference's forward (tests/test_oracle_golden.py) — and its eval-mode generator
  images, discriminator outputs / latents and aux-regressor coordinates equal the HIP path's
  eval-mode outputs of the same checkpoint within 1e-4 relative (fp32 mode).
"""
import os

import numpy as np
import pytest
import torch

from golden_utils import Golden

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLDEN_FOR = {"neutron": "neutron_e3_b12", "proton": "proton_e3_b12"}


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-6))


def _train_and_save(arch, tmp, E=2, steps=2, B=48):
    from expertsim.config import inject_shared, load_config
    from expertsim.train.loop import setup_moe_system
    from expertsim.train.training_setup import setup_optimizers
    from expertsim.train.training_utils import save_checkpoint
    from expertsim.utils.synthetic import make_batch
    shape = "[44,44]" if arch == "neutron" else "[56,30]"
    cfg = inject_shared(load_config(overrides=[f"model.architecture={arch}", f"model.n_experts={E}",
                                               "train.precision=fp32", "train.rng_seed=77",
                                               "model.router.diff_strength=1e-6",
                                               f"dataset.input_image_shape={shape}"]))
    torch.manual_seed(77)
    moe = setup_moe_system(cfg, torch.device(DEV))
    og, od, oa, orr = setup_optimizers(moe, cfg)
    for s in range(steps):
        b = make_batch(B, arch, seed=300 + s)
        t = lambda k: torch.from_numpy(b[k]).to(DEV)
        moe.train_step(0, t("cond"), t("real_images").unsqueeze(1), t("true_positions"), t("std"), t("intensity"),
                       oa, og, od, orr, None, DEV)
    torch.cuda.synchronize()
    save_checkpoint(str(tmp), 1, moe, og, od, oa, orr)
    return moe, cfg


@pytest.mark.parametrize("arch", ["neutron", "proton"])
def test_checkpoint_keys_are_the_reference_state_dict_keys(arch, tmp_path):
    g = Golden(GOLDEN_FOR[arch])
    moe, cfg = _train_and_save(arch, tmp_path, E=g.E)      # the router's shapes follow E
    ref_keys = {c: {k.split("/", 2)[2] for k in g.keys(f"init/{c}/")} for c in "GDAR"}
    files = {"G": "gen_0", "D": "disc_0", "A": "aux_reg_0", "R": "router_network"}
    for comp, stem in files.items():
        sd = torch.load(os.path.join(tmp_path, f"{stem}_epoch_1.pth"), map_location="cpu", weights_only=True)
        assert set(sd) == ref_keys[comp], (comp, set(sd) ^ ref_keys[comp])
        # shapes: the golden's per-tensor checksum holds 64 strided samples of numel >= 64
        for k, v in sd.items():
            ck = g[f"init/{comp}/{k}"]
            assert ck.shape == (3 + min(64, v.numel()),), (comp, k, v.shape)


@pytest.mark.parametrize("arch", ["neutron", "proton"])
def test_checkpoint_loads_into_the_oracle(arch, tmp_path):
    from oracle import expertsim_oracle as O
    moe, cfg = _train_and_save(arch, tmp_path)
    load = lambda stem: {k: v.float() if v.is_floating_point() else v for k, v in
                         torch.load(os.path.join(tmp_path, f"{stem}_epoch_1.pth"), map_location="cpu",
                                    weights_only=True).items()}
    gen = torch.Generator().manual_seed(5)
    B = 24
    noise = torch.randn(B, 10, generator=gen)
    cond = torch.randn(B, 9, generator=gen)
    for e in range(moe.n_experts):
        PG, PD, PA = load(f"gen_{e}"), load(f"disc_{e}"), load(f"aux_reg_{e}")
        G, D, A = moe.generators[e], moe.discriminators[e], moe.aux_regs[e]
        for m in (G, D, A):
            m.eval()
        with torch.no_grad():
            img = G(noise.to(DEV), cond.to(DEV)).cpu()
            out, lat = (t.cpu() for t in D(img.to(DEV), cond.to(DEV)))
            coords = A(img.to(DEV)).cpu()
            oimg = O.generator_forward(arch, PG, noise, cond, training=False)
            oout, olat = O.discriminator_forward(arch, PD, img, cond, training=False)
            ocoords = O.aux_forward(arch, PA, img, training=False)
        errs = {"G": _rel(img, oimg), "D.out": _rel(out, oout), "D.latent": _rel(lat, olat), "A": _rel(coords, ocoords)}
        print(arch, e, errs)
        for k, v in errs.items():
            assert v <= 1e-4, (arch, e, k, v)
