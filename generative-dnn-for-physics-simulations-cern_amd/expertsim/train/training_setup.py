"""Optimizer setup — reference: expertsim/train/training_setup.py:12-41.

One Adam per generator / discriminator / aux regressor and one for the router, with the
per-component learning rates of the config; here each is a FusedAdam over the module's flat
parameter buffer (expertsim/optim.py)."""
from __future__ import annotations

from ..optim import FusedAdam


def count_model_parameters(model):
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def setup_optimizers(wrapper, cfg):
    gen_optims = [FusedAdam(g, lr=cfg.model.generator.lr_g) for g in wrapper.generators]
    disc_optims = [FusedAdam(d, lr=cfg.model.discriminator.lr_d) for d in wrapper.discriminators]
    aux_reg_optims = [FusedAdam(a, lr=cfg.model.aux_reg.lr_a) for a in wrapper.aux_regs]
    router_optim = FusedAdam(wrapper.router, lr=cfg.model.router.lr_r)
    return gen_optims, disc_optims, aux_reg_optims, router_optim
