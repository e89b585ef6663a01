"""Data pipeline against goldens captured from the reference's own
get_dataset + transform_data_for_training (tests/golden/make_data_goldens.py): same pickled
inputs, same numpy seed → the same filtered / subsampled / paired / scaled / split arrays."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))

from expertsim.config import AttrDict  # noqa: E402
from expertsim.utils import data_transformations as DT  # noqa: E402

GOLD = np.load(os.path.join(ROOT, "tests", "golden", "data_pipeline.npz"))
META = json.loads(str(GOLD["meta"]))
OUT_NAMES = ["x_train", "x_test", "x2_train", "x2_test", "cond_train", "cond_test", "std_train", "std_test",
             "intensity_train", "intensity_test", "pos_train", "pos_test", "expert_train", "expert_test"]


def _write_case(tmp, name, zdc):
    import pandas as pd
    g = lambda k: GOLD[f"{name}/in/{k}"]
    cond = {c: g("cond")[:, i] for i, c in enumerate(DT.COND_COLUMNS)}
    if zdc == "proton":
        cond.update({"std_proton": g("std"), "proton_photon_sum": g("photon_sum"),
                     "group_number_proton": g("group"), "expert_number": g("expert_number")})
    else:
        cond.update({"std": g("std"), "neutron_photon_sum": g("photon_sum"), "group_number": g("group")})
    paths = [str(tmp / f) for f in ("images.pkl", "cond.pkl", "pos.pkl")]
    pd.to_pickle(g("images"), paths[0])
    pd.DataFrame(cond).to_pickle(paths[1])
    pd.DataFrame({"max_x": g("pos")[:, 0], "max_y": g("pos")[:, 1]}).to_pickle(paths[2])
    return paths


def _cfg(m, paths, tmp, source="pickle"):
    A = AttrDict
    return A(limit_samples=m["limit_samples"],
             config=A(run_name="t", experiment_dir=str(tmp / "exp")),
             model=A(architecture=m["zdc"]),
             dataset=A(zdc_type=m["zdc"], source=source, DATA_IMAGES_PATH=paths[0], DATA_COND_PATH=paths[1],
                       DATA_POSITIONS_PATH=paths[2], MIN_INTENSITY_THRESHOLD=m["MIN"],
                       MAX_INTENSITY_THRESHOLD=m["MAX"], read_n_samples=m["read_n_samples"],
                       shuffle_train_test_split=m["shuffle"], test_size=0.2, resident=False,
                       input_image_shape=[6, 5]),
             train=A(save_experiments_dir=str(tmp), checkpoint_experiment_dir=None, epoch_to_load=None,
                     save_experiment_data=False, batch_size=16))


@pytest.mark.parametrize("name", sorted(META))
def test_pipeline_matches_reference(tmp_path, name):
    m = META[name]
    cfg = _cfg(m, _write_case(tmp_path, name, m["zdc"]), tmp_path)
    np.random.seed(m["seed"])
    data, data_cond, data_posi = DT.get_dataset(cfg)
    out = DT.transform_data_for_training(cfg, data, data_cond, data_posi)
    for k, v in zip(OUT_NAMES, out[:14]):
        want = GOLD[f"{name}/out/{k}"]
        assert np.asarray(v).shape == want.shape, k
        np.testing.assert_array_equal(np.asarray(v), want, err_msg=f"{name}:{k}")   # bit-exact
    assert list(out[15]) == m["names"]
    assert cfg.photon_sum_min == m["photon_sum_min"] and cfg.photon_sum_max == m["photon_sum_max"]


def test_partner_pairing_properties():
    """Every partner has exactly the same conditioning values; a unique condition pairs with itself."""
    import pandas as pd
    rng = np.random.default_rng(0)
    vals = rng.integers(0, 3, size=(50, 9)).astype(float)
    vals[0] = 99.0
    df = pd.DataFrame(vals, columns=DT.COND_COLUMNS)
    np.random.seed(3)
    p = DT.same_condition_partners(df)
    assert p[0] == 0
    np.testing.assert_array_equal(vals[p], vals)


def test_save_and_reload_split(tmp_path):
    """save_experiment_data writes the reference's scales file + train_test_indices.npz; a resumed
    run (checkpoint_experiment_dir + epoch_to_load) reloads the same split."""
    name = "neutron_basic"
    m = META[name]
    paths = _write_case(tmp_path, name, m["zdc"])
    cfg = _cfg(m, paths, tmp_path)
    cfg.train.save_experiment_data = True
    np.random.seed(m["seed"])
    first = DT.transform_data_for_training(cfg, *DT.get_dataset(cfg))
    info = cfg.train.dir_info
    assert open(info + "neutron_scales.txt").read().startswith("#means\n")
    cfg2 = _cfg(m, paths, tmp_path)
    cfg2.config.experiment_dir = os.path.relpath(str(tmp_path / "exp"), str(tmp_path))
    cfg2.train.checkpoint_experiment_dir = str(tmp_path)
    cfg2.train.epoch_to_load = 3
    np.random.seed(m["seed"])
    second = DT.transform_data_for_training(cfg2, *DT.get_dataset(cfg2))
    assert len(second) == 15
    for a, b in zip(first[:2], second[:2]):
        np.testing.assert_array_equal(a, b)


def test_loaders_shard_by_rank(tmp_path):
    name = "proton_uniform"
    m = META[name]
    paths = _write_case(tmp_path, name, m["zdc"])
    shards = []
    for rank in range(2):
        cfg = _cfg(m, paths, tmp_path)
        np.random.seed(m["seed"])
        tr, te = DT.get_train_test_data_loaders(cfg, rank, 2)
        batches = list(tr)
        assert len(batches[0]) == 6 and batches[0][0].shape == (16, 6, 5) and batches[0][2].shape == (16, 9)
        shards.append(np.concatenate([b[0].numpy() for b in batches]))
    whole = GOLD[f"{name}/out/x_train"]
    np.testing.assert_array_equal(shards[0][:len(shards[0])], whole[0::2][:len(shards[0])])
    np.testing.assert_array_equal(shards[1][:len(shards[1])], whole[1::2][:len(shards[1])])


@pytest.mark.gpu
def test_resident_loader_on_device(tmp_path):
    """dataset.resident: the rank's shard is uploaded once; batches are HBM slices equal to the split."""
    import torch
    name = "neutron_basic"
    m = META[name]
    cfg = _cfg(m, _write_case(tmp_path, name, m["zdc"]), tmp_path)
    cfg.dataset.resident = True
    np.random.seed(m["seed"])
    tr, te = DT.get_train_test_data_loaders(cfg, 0, 1)
    assert isinstance(tr, DT.ResidentLoader)
    batches = list(tr)
    n_train = len(GOLD[f"{name}/out/x_train"])
    # one device keeps the last partial batch, as the reference's DataLoader (drop_last=False)
    assert len(batches) == -(-n_train // 16)
    assert batches[-1][0].shape[0] == (n_train % 16 or 16)
    assert all(t.is_cuda for t in batches[0])
    got = torch.cat([b[0] for b in batches]).cpu().numpy()
    np.testing.assert_array_equal(got, GOLD[f"{name}/out/x_train"])
    assert sum(b[0].shape[0] for b in te) == len(GOLD[f"{name}/out/x_test"])
