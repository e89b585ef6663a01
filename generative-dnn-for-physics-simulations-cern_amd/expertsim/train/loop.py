"""Training orchestration — reference: expertsim/train/loop.py:27-182,332-354.

Same entry points (``train``, ``train_epoch``, ``train_step``, ``setup_moe_system``); the per-batch
step is ``MoEWrapper.train_step`` on the HIP path.  Metrics are fetched to the host once per batch
(the reference does ``.cpu().item()`` per key, loop.py:136-148).  With WORLD_SIZE > 1 (torchrun),
every rank trains on its own shard and gradients are all-reduced over RCCL (expertsim/train/ddp.py).
``evaluate_epoch`` (loop.py:185-256) produces the Wasserstein metrics of MoEWrapper.evaluate on the
HIP path.  Checkpoints (hooks.CheckpointSaver, training_utils) and the
EMAHelper (ema.py) follow loop.py:36-107,357-418; resume restores weights, optimizer moments and
the step counters.  Plotting and W&B stay out of scope.
"""
from __future__ import annotations

import logging
import os
import time
from typing import Dict, List

import numpy as np
import torch

from ..models import build_model
from ..models.moe import MoEWrapper
from .ema import EMAHelper
from .hooks import CheckpointSaver
from .training_setup import setup_optimizers
from .training_utils import load_checkpoint

logger = logging.getLogger(__name__)


def setup_moe_system(cfg, device) -> MoEWrapper:
    from ..config import inject_shared
    inject_shared(cfg)
    generator = build_model(f"{cfg.model.architecture}.generator", cfg.model.generator, device)
    discriminator = build_model(f"{cfg.model.architecture}.discriminator", cfg.model.discriminator, device)
    aux_reg = build_model(f"{cfg.model.architecture}.aux_reg", cfg.model.aux_reg, device)
    router = build_model(f"{cfg.model.router.version}", cfg.model.router, device)
    return MoEWrapper(generator, discriminator, aux_reg, router, cfg.model.n_experts, cfg,
                      image_shape=tuple(cfg.dataset.input_image_shape)).to(device)


def train_step(batch, moe, gen_optims, disc_optims, aux_reg_optim, router_optim, cfg, device, epoch,
               ema_helper) -> Dict:
    real_images, _, cond, std, intensity, true_positions = batch
    real_images = real_images.unsqueeze(1).to(device, non_blocking=True)
    return moe.train_step(epoch, cond.to(device, non_blocking=True), real_images,
                          true_positions.to(device, non_blocking=True), std.to(device, non_blocking=True),
                          intensity.to(device, non_blocking=True), aux_reg_optim, gen_optims, disc_optims,
                          router_optim, ema_helper, device)


def setup_callbacks(cfg, moe, ema_helper=None) -> List:
    """loop.py:357-375 (the W&B logger is out of scope)."""
    callbacks = []
    cfg.generator_name = getattr(moe.generators[0], "name", "generator")
    cfg.discriminator_name = getattr(moe.discriminators[0], "name", "discriminator")
    cfg.router_name = getattr(moe.router, "name", "router")
    if cfg.train.get("save_experiment_data", False):
        callbacks.append(CheckpointSaver(dir_path=_dir_models(cfg), monitor="ws_mean",
                                         ws_threshold=cfg.train.ws_threshold_model_save, ema_helper=ema_helper))
    return callbacks


def _dir_models(cfg):
    d = cfg.train.get("dir_models")
    if d is None:
        exp = cfg.get_path("config.experiment_dir") or os.path.join(cfg.train.get("save_experiments_dir") or "",
                                                                     cfg.config.get("run_name", "experiment"))
        d = cfg.train.dir_models = f"{exp}/models/"
    return d


def train_epoch(moe, train_loader, gen_optims, disc_optims, aux_reg_optims, router_optim, cfg, device, epoch,
                ema_helper, max_steps=None) -> Dict:
    moe.train()
    sums: Dict[str, List[float]] = {}
    for i, batch in enumerate(train_loader):
        if max_steps is not None and i >= max_steps:
            break
        m = train_step(batch, moe, gen_optims, disc_optims, aux_reg_optims, router_optim, cfg, device, epoch,
                       ema_helper)
        if ema_helper is not None and cfg.train.get("ema_update", False):
            ema_helper.update(moe, range(moe.n_experts))     # build extension: the reference never updates
        keys = list(m)
        vals = torch.stack([torch.as_tensor(m[k], dtype=torch.float32, device=device).reshape(())
                            for k in keys]).cpu().numpy()   # ONE device->host copy per batch
        for k, v in zip(keys, vals):
            sums.setdefault(k, []).append(float(v))
    out = {k: float(np.mean(v)) for k, v in sums.items()}
    for i in range(moe.n_experts):
        out[f"G_steps_{i}"] = moe.g_steps[i]
        out[f"D_steps_{i}"] = moe.d_steps[i]
    return out


@torch.no_grad()
def evaluate_epoch(moe, test_loader, epoch: int, cfg, device, max_batches=None) -> Dict:
    """Reference loop.py:185-256 without the plots: per-batch MoEWrapper.evaluate, averaged."""
    moe.eval()
    keys = ["ws_mean", *[f"ws_mean_{i}" for i in range(moe.n_experts)],
            "ws_std", *[f"ws_std_{i}" for i in range(moe.n_experts)]]
    acc: Dict[str, List[float]] = {k: [] for k in keys}
    for b, batch in enumerate(test_loader):
        if max_batches is not None and b >= max_batches:
            break
        real_images, _, cond, std, intensity, true_positions = batch
        m = moe.evaluate(epoch, cond.to(device), real_images, true_positions, std, intensity, cfg, device)
        for k in keys:
            acc[k].append(float(m[k]))
    return {k: (sum(v) / len(v) if v else 0.0) for k, v in acc.items()}


def train(cfg, train_loader, test_loader=None, max_steps_per_epoch=None) -> List[Dict]:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise RuntimeError("expertsim trains on a HIP device only (no CPU fallback)")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    torch.manual_seed(int(cfg.train.get("rng_seed", 1234)))
    moe = setup_moe_system(cfg, device)
    if world > 1:
        import torch.distributed as dist
        from .ddp import DataParallel
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("nccl", device_id=device)
        moe.ddp = DataParallel(sync_bn=bool(cfg.train.get("sync_bn", False)))
        moe.rank = dist.get_rank()
    gen_optims, disc_optims, aux_optims, router_optim = setup_optimizers(moe, cfg)
    ema_helper = EMAHelper(moe, decay=0.99)                 # loop.py:44
    history = []
    start = 0
    ckpt_dir, ckpt_epoch = cfg.train.get("checkpoint_experiment_dir"), cfg.train.get("epoch_to_load")
    if (ckpt_dir is None) != (ckpt_epoch is None):
        raise ValueError("You should set both checkpoint_experiment_dir and epoch_to_load parameters!")
    if ckpt_dir is not None:
        load_checkpoint(os.path.join(ckpt_dir, "models"), int(ckpt_epoch), moe, gen_optims, disc_optims, aux_optims,
                        router_optim, ema_helper, device)
        start = int(ckpt_epoch) + 1
    callbacks = setup_callbacks(cfg, moe, ema_helper if cfg.train.get("ema_update", False) else None)
    for epoch in range(start, int(cfg.train.epochs)):
        t0 = time.time()
        metrics = train_epoch(moe, train_loader, gen_optims, disc_optims, aux_optims, router_optim, cfg, device,
                              epoch, ema_helper, max_steps=max_steps_per_epoch)
        if test_loader is not None:
            metrics.update(evaluate_epoch(moe, test_loader, epoch, cfg, device))
        for cb in callbacks:
            if moe.rank == 0:
                cb.on_epoch_end(epoch, metrics, moe, gen_optims, disc_optims, aux_optims, router_optim)
        metrics["epoch_time"] = time.time() - t0
        metrics["epoch"] = epoch
        history.append(metrics)
        logger.info("Epoch %d: %.2fs gen_loss %.4f disc_loss %.4f", epoch, metrics["epoch_time"],
                    metrics.get("gen_loss", float("nan")), metrics.get("disc_loss", float("nan")))
    return history
