"""Batch sources — reference: expertsim/utils/data_transformations.py:23-309.

``get_train_test_data_loaders(cfg, rank, world)`` returns (train_loader, test_loader) yielding the
reference's 6-tuples ``(real_images [B,H,W], real_images_2, cond [B,9], std [B,1],
intensity [B,1], true_positions [B,2])`` (consumed at expertsim/train/loop.py:170).

Two sources (``dataset.source``):

* ``synthetic`` (default): the seeded synthetic ZDC batches of expertsim/utils/synthetic.py (the
  reference ships no data);
* ``pickle``: the reference's on-disk format — the three pandas pickles named by
  ``DATA_IMAGES_PATH`` (images [N,H,W], log1p domain), ``DATA_COND_PATH`` (DataFrame: the 9
  conditioning columns Energy, Vx, Vy, Vz, Px, Py, Pz, mass, charge, plus ``std``/``std_proton``,
  ``neutron_photon_sum``/``proton_photon_sum``, ``group_number``/``group_number_proton`` and, for
  protons, ``expert_number``) and ``DATA_POSITIONS_PATH`` (DataFrame with ``max_x``, ``max_y``).
  ``get_dataset`` and ``transform_data_for_training`` follow the reference's filtering,
  photon-sum-uniform subsampling, same-condition partner pairing, scaling and train/test split,
  consuming numpy's global RNG in the reference's order, so a seeded run selects the same
  samples (pinned by tests/golden/data_pipeline.npz, captured from the reference's functions).
  Only load pickles you produced yourself: unpickling executes code from the file.

MI355X-first: the split dataset is small (N·H·W·4 bytes, ~2.3 GB for 300 k neutron images), so
with ``dataset.resident: true`` (the default) each rank's shard is copied to HBM once and batches
are device slices — no per-step host→device copy or pinned staging.  With ``world > 1`` each rank
takes the strided shard ``rank::world`` of the training set (DistributedSampler order, no shuffle,
as the reference's loaders have ``shuffle=False``).
"""
from __future__ import annotations

import logging
import os
from enum import Enum

import numpy as np
import torch
from torch.utils.data import DataLoader, TensorDataset

from .synthetic import make_batch

logger = logging.getLogger(__name__)

COND_COLUMNS = ["Energy", "Vx", "Vy", "Vz", "Px", "Py", "Pz", "mass", "charge"]
TRAIN_TEST_INDICES_FILENAME = "train_test_indices.npz"     # expertsim/utils/utils.py:9


class ZDCType(Enum):
    PROTON = "proton"
    NEUTRON = "neutron"


def _photon_sum_column(zdc_type: str) -> str:
    return "proton_photon_sum" if zdc_type == ZDCType.PROTON.value else "neutron_photon_sum"


def _opt(node, key, default=None):
    try:
        v = node[key] if isinstance(node, dict) else getattr(node, key)
    except (KeyError, AttributeError):
        return default
    return default if v is None else v


# ---------------------------------------------------------------------------------------------
# reading + filtering (data_transformations.py:23-129)
# ---------------------------------------------------------------------------------------------

def _keep_rows(mask, data, data_cond, data_posi):
    mask = np.asarray(mask, dtype=bool)
    return (data[mask], data_cond[mask].reset_index(drop=True), data_posi[mask].reset_index(drop=True))


def _photon_sum_uniform_indices(values, n_samples: int, n_bins: int = 1000):
    """data_transformations.py:72-107: up to max(1, n/n_bins) samples from each photon-sum
    quantile bin (np.random.choice without replacement), topped up uniformly from the rest."""
    import pandas as pd
    bins = pd.qcut(values, q=n_bins, duplicates="drop")
    per_bin = max(1, n_samples // n_bins)
    chosen = []
    for interval in bins.unique():
        members = values.index[np.asarray(bins == interval)].to_list()
        chosen.extend(np.random.choice(members, size=min(per_bin, len(members)), replace=False))
    if len(chosen) < n_samples:
        rest = list(set(values.index) - set(chosen))
        chosen.extend(np.random.choice(rest, size=n_samples - len(chosen), replace=False))
    return np.array(chosen)


def get_dataset(cfg):
    """Reference get_dataset (data_transformations.py:23-129) → (images ndarray [N,H,W],
    cond DataFrame, positions DataFrame); sets cfg.photon_sum_min / photon_sum_max."""
    import pandas as pd
    ds = cfg.dataset
    limit = _opt(cfg, "limit_samples")
    frames = [pd.read_pickle(ds[k]) for k in ("DATA_IMAGES_PATH", "DATA_COND_PATH", "DATA_POSITIONS_PATH")]
    if limit is not None:
        frames = [f[:int(limit)] for f in frames]
    data, data_cond, data_posi = frames
    data = np.asarray(data)
    ps_col = _photon_sum_column(ds.zdc_type)

    lo, hi = _opt(ds, "MIN_INTENSITY_THRESHOLD"), _opt(ds, "MAX_INTENSITY_THRESHOLD")
    if lo is not None:
        logger.info("Filtering data with min intensity threshold: %s", lo)
        data, data_cond, data_posi = _keep_rows(data_cond[ps_col] >= lo, data, data_cond, data_posi)
    if hi is not None:
        logger.info("Filtering data with max intensity threshold: %s", hi)
        data, data_cond, data_posi = _keep_rows(data_cond[ps_col] <= hi, data, data_cond, data_posi)

    n_samples = _opt(ds, "read_n_samples")
    if n_samples is not None:
        idx = _photon_sum_uniform_indices(data_cond[ps_col], int(n_samples))
        data = data[idx]
        data_cond = data_cond.loc[idx].reset_index(drop=True)
        data_posi = data_posi.loc[idx].reset_index(drop=True)
        logger.info("Sampling %d uniform samples based on photon_sum distribution.", int(n_samples))

    cfg.photon_sum_min = float(data_cond[ps_col].min())
    cfg.photon_sum_max = float(data_cond[ps_col].max())
    logger.info("Photon sum min: %s, max: %s", cfg.photon_sum_min, cfg.photon_sum_max)
    return data, data_cond, data_posi


# ---------------------------------------------------------------------------------------------
# transformation + split (data_transformations.py:131-257)
# ---------------------------------------------------------------------------------------------

def same_condition_partners(data_cond):
    """data_transformations.py:151-161: every sample's partner is the first sample, in one
    shuffled order of all rows (``DataFrame.sample(frac=1)``, global numpy RNG), whose 9
    conditioning values print identically.  Returns the partner index per row."""
    import pandas as pd
    data_cond = data_cond.reset_index(drop=True)
    key = data_cond[COND_COLUMNS[0]].astype(str)
    for c in COND_COLUMNS[1:]:
        key = key + "|" + data_cond[c].astype(str)
    codes, _ = pd.factorize(key.to_numpy())
    order = data_cond.reset_index()[["index"]].sample(frac=1)["index"].to_numpy()
    shuffled = codes[order]
    _, first_pos = np.unique(shuffled, return_index=True)     # first occurrence of each key
    partner_of_code = np.empty(len(first_pos), dtype=np.int64)
    partner_of_code[np.unique(shuffled)] = order[first_pos]
    return partner_of_code[codes]


def _scales_text(means, scales):
    """expertsim/utils/utils.py:29-39 file format."""
    return "#means" + "".join(f"\n{m}" for m in means) + "\n\n#scales" + "".join(f"\n{s}" for s in scales)


def transform_data_for_training(cfg, data, data_cond, data_posi):
    """Reference transform_data_for_training (data_transformations.py:131-257).  Returns the same
    tuple: x, x_2, cond, std, intensity, positions (train/test each), expert numbers (train/test),
    the (unused) position scaler, the conditioning column names and the models directory."""
    from sklearn.model_selection import train_test_split
    from sklearn.preprocessing import MinMaxScaler, StandardScaler
    zdc = cfg.dataset.zdc_type
    root = cfg.train.get("save_experiments_dir") or ""
    exp = cfg.get_path("config.experiment_dir") if hasattr(cfg, "get_path") else None
    exp = exp or cfg.config.get("run_name", "experiment")
    if cfg.train.get("checkpoint_experiment_dir") is not None:
        exp = os.path.join(root, exp)
    dir_info, dir_models = f"{exp}/info/", f"{exp}/models/"
    cfg.train.dir_info, cfg.train.dir_models = dir_info, dir_models

    partners = same_condition_partners(data_cond)
    data = data.astype(np.float32)
    data_2 = data[partners]
    indices = np.arange(len(data))

    if zdc == ZDCType.PROTON.value:
        expert_number = data_cond["expert_number"].to_numpy()
        std_col, drop = "std_proton", ["std_proton", "proton_photon_sum", "group_number_proton", "expert_number"]
    elif zdc == ZDCType.NEUTRON.value:
        expert_number = None
        std_col, drop = "std", ["std", "neutron_photon_sum", "group_number"]
    else:
        raise ValueError("Unsupported ZDC type! Choose either proton or neutron.")
    std = MinMaxScaler().fit_transform(np.float32(data_cond[std_col].to_numpy().reshape(-1, 1)))
    intensity = np.float32(data_cond[_photon_sum_column(zdc)].to_numpy().reshape(-1, 1))
    cond_frame = data_cond.drop(columns=drop)
    positions = np.float32(data_posi[["max_x", "max_y"]].to_numpy())   # not scaled (reference :198)
    scaler_pos = StandardScaler()
    names = cond_frame.columns
    scaler_cond = StandardScaler()
    cond = scaler_cond.fit_transform(cond_frame.astype(np.float32))

    ckpt, epoch = cfg.train.get("checkpoint_experiment_dir"), cfg.train.get("epoch_to_load")
    if ckpt and epoch:
        f = np.load(os.path.join(dir_info, TRAIN_TEST_INDICES_FILENAME))
        tr, te = f["train_indices"], f["test_indices"]
        arrays = [data, data_2, cond, std, intensity, positions]
        out = []
        for a in arrays:
            out += [a[tr], a[te]]
        return (*out, scaler_pos, names, dir_models)
    if (ckpt is None) != (epoch is None):
        raise ValueError("You should set both checkpoint_experiment_dir and epoch_to_load parameters!")

    arrays = [data, data_2, cond, std, intensity, positions]
    if expert_number is not None:
        arrays.append(expert_number)
    split = train_test_split(*arrays, indices, test_size=cfg.dataset.test_size,
                             shuffle=cfg.dataset.shuffle_train_test_split)
    tr_idx, te_idx = split[-2], split[-1]
    if expert_number is not None:
        en_tr, en_te = split[12], split[13]
    else:
        en_tr, en_te = np.zeros(len(tr_idx)), np.zeros(len(te_idx))
    if cfg.train.get("save_experiment_data"):
        os.makedirs(dir_info, exist_ok=True)
        with open(dir_info + f"{zdc}_scales.txt", "w") as fh:
            fh.write(_scales_text(scaler_cond.mean_, scaler_cond.scale_))
        os.makedirs(dir_models, exist_ok=True)
        np.savez(os.path.join(dir_info, TRAIN_TEST_INDICES_FILENAME), train_indices=tr_idx, test_indices=te_idx)
    else:
        dir_models = None
    return (*split[:12], en_tr, en_te, scaler_pos, names, dir_models)


# ---------------------------------------------------------------------------------------------
# loaders (data_transformations.py:260-309)
# ---------------------------------------------------------------------------------------------

class ResidentLoader:
    """Batches as slices of tensors already in HBM (one upload per rank, no per-step H2D).
    Same iteration contract as the reference's DataLoader(shuffle=False)."""

    def __init__(self, tensors, batch_size: int, drop_last: bool):
        self.tensors = tensors
        self.batch_size = int(batch_size)
        self.drop_last = drop_last
        self.n = int(tensors[0].shape[0])

    def __len__(self):
        return self.n // self.batch_size if self.drop_last else -(-self.n // self.batch_size)

    def __iter__(self):
        for i in range(len(self)):
            s = slice(i * self.batch_size, min((i + 1) * self.batch_size, self.n))
            yield tuple(t[s] for t in self.tensors)


def _make_loader(tensors, bs, drop_last, resident, device):
    if resident:
        return ResidentLoader([t.to(device) for t in tensors], bs, drop_last)
    return DataLoader(TensorDataset(*tensors), batch_size=bs, shuffle=False, drop_last=drop_last,
                      pin_memory=torch.cuda.is_available())


def _shard(tensors, rank, world):
    if world <= 1:
        return tensors
    n = (tensors[0].shape[0] // world) * world                  # DistributedSampler(drop_last=True)
    return [t[rank:n:world] for t in tensors]


def _synthetic_sets(cfg, rank):
    arch = cfg.model.architecture
    n = int(cfg.dataset.get("synthetic_samples", 4096))
    n_test = int(n * float(cfg.dataset.get("test_size", 0.2)))
    shape = tuple(cfg.dataset.input_image_shape)
    sets = []
    for count, seed in ((n - n_test, 1000 + rank), (max(n_test, 1), 999_000 + rank)):
        b = make_batch(count, arch, seed=seed, shape=shape)
        x = torch.from_numpy(b["real_images"])
        sets.append([x, x, torch.from_numpy(b["cond"]), torch.from_numpy(b["std"]),
                     torch.from_numpy(b["intensity"]), torch.from_numpy(b["true_positions"])])
    return sets


def _pickle_sets(cfg, rank, world):
    data, data_cond, data_posi = get_dataset(cfg)
    out = transform_data_for_training(cfg, data, data_cond, data_posi)
    cfg.data_cond_names = list(out[-2])
    to_t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
    train = [to_t(out[i]) for i in (0, 2, 4, 6, 8, 10)]
    test = [to_t(out[i]) for i in (1, 3, 5, 7, 9, 11)]
    return _shard(train, rank, world), test


def get_train_test_data_loaders(cfg, rank: int = 0, world: int = 1, device=None):
    """(train_loader, test_loader) for this rank.  Synthetic sets are generated per rank (seeded
    by rank); pickle sets are split once and sharded ``rank::world``."""
    source = cfg.dataset.get("source", "synthetic")
    if source == "synthetic":
        train, test = _synthetic_sets(cfg, rank)
    elif source == "pickle":
        train, test = _pickle_sets(cfg, rank, world)
    else:
        raise ValueError(f"dataset.source must be 'synthetic' or 'pickle', got {source!r}")
    bs = int(cfg.train.batch_size)
    resident = bool(cfg.dataset.get("resident", True)) and torch.cuda.is_available()
    if device is None and resident:
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    # the reference's DataLoader keeps the last partial batch (data_transformations.py:275,298);
    # data-parallel ranks drop it so every rank runs the same number of equal-sized steps
    return (_make_loader(train, bs, world > 1, resident, device),
            _make_loader(test, bs, False, resident, device))
