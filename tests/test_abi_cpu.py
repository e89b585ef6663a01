"""CPU-side checks of the C ABI library and host logic (no GPU needed)."""
import os
import re
import subprocess

import numpy as np
import torch
import torch.nn.functional as F

from conftest import PKG_DIR, REPO

HEADER = os.path.join(REPO, "include", "expertsim_hip.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(es_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_declared_symbol():
    from expertsim import hip
    lib = hip.lib()                       # loads without a GPU
    for name in _declared():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", hip.lib_path()], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (es_[a-z0-9_]+)", out))
    assert set(_declared()) <= exported
    assert set(hip._SIGS) <= exported
    assert lib.es_version() == 1


def test_library_is_built_for_gfx950():
    from expertsim import hip
    data = open(hip.lib_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_upsample_maps_match_torch_nearest():
    from expertsim.layers import Upsample
    for in_hw, kw in (((13, 13), dict(scale=(2, 2))), ((24, 24), dict(scale=(2, 2))),
                      ((18, 10), dict(scale=(2, 2))), ((35, 19), dict(out_hw=(56, 30)))):
        up = Upsample(in_hw, **kw)
        H, W = in_hw
        x = torch.arange(H * W, dtype=torch.float32).view(1, 1, H, W)
        if "scale" in kw:
            y = F.interpolate(x, scale_factor=kw["scale"], mode="nearest")
        else:
            y = F.interpolate(x, size=kw["out_hw"], mode="nearest")
        ours = x[0, 0][up.maps[0]][:, up.maps[1]]
        assert torch.equal(ours, y[0, 0])
        for ax in range(2):
            start, count = up.inv[ax]
            assert count.sum() == up.out_hw[ax]


def test_model_init_matches_reference_checksums():
    from golden_utils import Golden, checksum
    from expertsim.config import inject_shared, load_config
    from expertsim.models import build_model
    for case in ("neutron_e1_b8", "proton_e1_b8"):
        g = Golden(case)
        cfg = inject_shared(load_config(overrides=[f"model.architecture={g.arch}", f"model.n_experts={g.E}"]))
        torch.manual_seed(g.seed)
        comps = {"G": build_model(f"{g.arch}.generator", cfg.model.generator, "cpu"),
                 "D": build_model(f"{g.arch}.discriminator", cfg.model.discriminator, "cpu"),
                 "A": build_model(f"{g.arch}.aux_reg", cfg.model.aux_reg, "cpu"),
                 "R": build_model("router_v1", cfg.model.router, "cpu")}
        for comp, m in comps.items():
            sd = m.state_dict()
            assert set(sd) == {k.split("/", 2)[2] for k in g.keys(f"init/{comp}/")}
            for n, t in sd.items():
                np.testing.assert_array_equal(checksum(t.float().numpy()), g[f"init/{comp}/{n}"])


def test_config_schema_and_coercion():
    from expertsim.config import load_config
    cfg = load_config(overrides=["model.n_experts=4", "train.batch_size=64"])
    assert cfg.model.generator.lr_g == 1e-4 and isinstance(cfg.model.generator.lr_g, float)
    assert cfg.model.router.diff_strength == 1e-6
    assert cfg.model.n_experts == 4 and cfg.train.batch_size == 64


def test_product_fails_loudly_without_device():
    import pytest
    from expertsim import hip
    with pytest.raises(hip.HipError):
        hip.require_device(torch.zeros(1))
