"""cli.py end to end on the HIP path (reference cli.py:37-118 -> train/loop.py:27-182): the synthetic
data source, 2 epochs of a 3-expert neutron run (dynamic-rows multi-expert steps), the per-epoch
evaluation (Wasserstein metrics), a checkpoint per epoch, then a resume from epoch 1 for a third
epoch.  Checked: the reference's metric keys per epoch, every value finite, WS finite and > 0, the
checkpoint files, the resumed run starting at epoch 2 with the saved optimizer step counts."""
import glob
import math
import os
import sys

import pytest

pytestmark = pytest.mark.gpu


def _run_cli(argv):
    import cli
    from expertsim.train import loop
    hist = []
    orig = loop.train

    def train(*a, **k):
        out = orig(*a, **k)
        hist.extend(out)
        return out
    loop.train = train
    old = sys.argv
    sys.argv = ["cli.py", *argv]
    try:
        cli.main()
    finally:
        sys.argv = old
        loop.train = orig
    return hist


@pytest.mark.timeout(600)
def test_cli_two_epochs_checkpoint_resume(tmp_path):
    common = ["model.architecture=neutron", "dataset.input_image_shape=[44,44]", "model.n_experts=3",
              "train.batch_size=64", "dataset.synthetic_samples=640", "train.save_experiment_data=true",
              "train.ws_threshold_model_save=1e9", f"train.dir_models={tmp_path}/models/"]
    hist = _run_cli(["-o", *common, "train.epochs=2"])
    assert [h["epoch"] for h in hist] == [0, 1]
    keys = {"gen_loss", "disc_loss", "div_loss", "intensity_loss", "aux_reg_loss", "router_loss",
            "expert_distribution_loss", "differentiation_loss", "expert_entropy_loss",
            "adaptive_load_balancing_loss", "gan_loss", "ws_mean", "ws_std"}
    for i in range(3):
        keys |= {f"gen_loss_{i}", f"disc_loss_{i}", f"n_choosen_experts_mean_epoch_{i}", f"ws_mean_{i}",
                 f"ws_std_{i}"}
    for h in hist:
        assert keys <= set(h), sorted(keys - set(h))
        assert all(math.isfinite(float(v)) for v in h.values()), h
        assert h["ws_mean"] > 0.0
        assert sum(h[f"n_choosen_experts_mean_epoch_{i}"] for i in range(3)) == pytest.approx(64.0)
    saved = sorted(os.path.basename(p) for p in glob.glob(f"{tmp_path}/models/*.pth"))
    for ep in (0, 1):
        assert any(f"epoch_{ep}.pth" in s for s in saved), saved
    res = _run_cli(["-o", *common, "train.epochs=3", f"train.checkpoint_experiment_dir={tmp_path}",
                    "train.epoch_to_load=1"])
    assert [h["epoch"] for h in res] == [2]
    assert keys <= set(res[0]) and all(math.isfinite(float(v)) for v in res[0].values())
