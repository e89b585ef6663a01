"""Batch sources — reference: expertsim/utils/data_transformations.py:260-309.

``get_train_test_data_loaders(cfg)`` returns (train_loader, test_loader) yielding the reference's
6-tuples ``(real_images [B,H,W], real_images_2, cond [B,9], std [B,1], intensity [B,1],
true_positions [B,2])`` (consumed at expertsim/train/loop.py:170).  The reference reads GEANT4
pickles that do not ship with it; this build provides the seeded synthetic source of
expertsim/utils/synthetic.py (``dataset.source: synthetic``).  Reading the real pickles is a
"next" row of SURVEY.md §8(f) and is not implemented."""
from __future__ import annotations

import torch
from torch.utils.data import DataLoader, TensorDataset

from .synthetic import make_batch


def _dataset(n, arch, seed, shape=None):
    b = make_batch(n, arch, seed=seed, shape=shape)
    x = torch.from_numpy(b["real_images"])
    return TensorDataset(x, x, torch.from_numpy(b["cond"]), torch.from_numpy(b["std"]),
                         torch.from_numpy(b["intensity"]), torch.from_numpy(b["true_positions"]))


def get_train_test_data_loaders(cfg, rank: int = 0, world: int = 1):
    source = cfg.dataset.get("source", "synthetic") if isinstance(cfg.dataset, dict) else "synthetic"
    if source != "synthetic":
        raise NotImplementedError("only dataset.source=synthetic is available (the reference's pickles "
                                  "are not shipped); see SURVEY.md §8(f) row 2")
    arch = cfg.model.architecture
    n = int(cfg.dataset.get("synthetic_samples", 4096))
    n_test = int(n * float(cfg.dataset.get("test_size", 0.2)))
    shape = tuple(cfg.dataset.input_image_shape)
    train = _dataset(n - n_test, arch, seed=1000 + rank, shape=shape)
    test = _dataset(max(n_test, 1), arch, seed=999_000 + rank, shape=shape)
    bs = int(cfg.train.batch_size)
    return (DataLoader(train, batch_size=bs, shuffle=False, drop_last=True, pin_memory=True),
            DataLoader(test, batch_size=bs, shuffle=False, pin_memory=True))
