"""Training callbacks — reference: expertsim/train/hooks.py (Callback, CheckpointSaver :102-165).

``CheckpointSaver`` keeps the reference's constructor and ``on_epoch_end`` signature and its
rule: save when the monitored metric (``ws_mean``) is below the threshold.  What it writes is
described in expertsim/train/training_utils.py (state_dicts + training state, safe to load).
W&B logging (hooks.py:29-99) is out of scope (no network).
"""
from __future__ import annotations

import logging
from pathlib import Path
from typing import Dict

import torch

from .training_utils import save_checkpoint

logger = logging.getLogger(__name__)


class Callback:
    def on_epoch_end(self, epoch: int, metrics: Dict, moe, gen_optims, disc_optims, aux_reg_optim, router_optim):
        pass


class CheckpointSaver(Callback):
    def __init__(self, dir_path: str, ema_helper=None, monitor: str = "ws_mean", ws_threshold: float = 2.0):
        self.dir_path = Path(dir_path)
        self.monitor = monitor
        self.threshold = ws_threshold
        self.ema_helper = ema_helper
        self.dir_path.mkdir(parents=True, exist_ok=True)
        logger.info("Checkpoints will be saved to %s", self.dir_path)

    def on_epoch_end(self, epoch, metrics, moe, gen_optims, disc_optims, aux_reg_optim, router_optim):
        current = metrics.get(self.monitor, float("inf"))
        if not current < self.threshold:
            return False
        save_checkpoint(str(self.dir_path), epoch, moe, gen_optims, disc_optims, aux_reg_optim, router_optim,
                        self.ema_helper)
        logger.info("New best %s: %.4f at epoch %d", self.monitor, current, epoch)
        if self.ema_helper is not None:
            self.save_ema_weights(self.dir_path / f"ema_generators_epoch_{epoch}.pt", epoch=epoch)
        return True

    def save_ema_weights(self, save_path, epoch=None):
        """hooks.py:138-152 format: {'ema_shadow': {i: {name: tensor}}, 'decay', 'epoch'}."""
        save_path = Path(save_path)
        save_path.parent.mkdir(parents=True, exist_ok=True)
        shadow = {i: {k: v.detach().cpu().clone() for k, v in s.items()} for i, s in self.ema_helper.shadow.items()}
        torch.save({"ema_shadow": shadow, "decay": self.ema_helper.decay, "epoch": epoch}, save_path)

    def load_ema_weights(self, load_path, moe):
        """hooks.py:154-165: copy the saved EMA weights into the generators."""
        ckpt = torch.load(load_path, map_location="cpu", weights_only=True)
        for i, gen in enumerate(moe.generators):
            with torch.no_grad():
                for name, p in gen.named_parameters():
                    if p.requires_grad:
                        p.copy_(ckpt["ema_shadow"][i][name].to(p.device))
            gen.invalidate()
        logger.info("[EMA] Loaded EMA weights from %s (epoch %s)", load_path, ckpt.get("epoch"))
