"""Checkpoint save / resume — reference: save_models_and_architectures
(expertsim/train/training_utils.py:316-381) and the intended load_checkpoint_weights
(expertsim/train/training_setup.py:70-214).

File names follow the reference: ``{gen,disc,aux_reg}_{i}_epoch_{e}.pth``,
``{gen,disc,aux_reg}_optim_{i}_epoch_{e}.pth``, ``router_network_epoch_{e}.pth``,
``router_network_optim_epoch_{e}.pth``.  Deliberate differences:

* the reference ``torch.save``s whole modules and optimizers (pickled objects, loadable only with
  ``weights_only=False``); here every file holds a ``state_dict`` of tensors and plain values, so
  loading uses ``torch.load(..., weights_only=True)`` — nothing in a checkpoint is executed;
* the reference's resume never loads weights (and looks for ``gen_{i}_{epoch}.pth``, a name it
  never writes); here ``load_checkpoint_weights`` restores models (parameters, BatchNorm running
  statistics, spectral-norm u/v), fused-Adam moments and step counts;
* ``train_state_epoch_{e}.pth`` adds what a bit-faithful resume needs on this build: the MoE step
  counter (keys the device dropout / noise / Gumbel Philox streams), per-expert G/D step counts,
  the Philox seed and device RNG stream counter, and the EMA shadow when one is kept.
"""
from __future__ import annotations

import os

import torch


def _path(d, name, epoch, idx=None):
    return os.path.join(d, f"{name}_epoch_{epoch}.pth" if idx is None else f"{name}_{idx}_epoch_{epoch}.pth")


def _sd(x):
    return x.state_dict() if hasattr(x, "state_dict") else x


def save_models_and_architectures(filepath_models, n_experts, aux_regs, aux_reg_optimizers, generators,
                                  generator_optimizers, discriminators, discriminator_optimizers, router_network,
                                  router_optimizer, epoch, multiple_aux_regs=False):
    os.makedirs(filepath_models, exist_ok=True)
    groups = [("gen", generators, generator_optimizers), ("disc", discriminators, discriminator_optimizers)]
    groups.insert(0, ("aux_reg", aux_regs if multiple_aux_regs else list(aux_regs)[:1],
                      aux_reg_optimizers if multiple_aux_regs else list(aux_reg_optimizers)[:1]))
    for name, mods, opts in groups:
        for i, m in enumerate(list(mods)[:n_experts]):
            torch.save(_sd(m), _path(filepath_models, name, epoch, i))
        for i, o in enumerate(list(opts)[:n_experts]):
            torch.save(_sd(o), _path(filepath_models, f"{name}_optim", epoch, i))
    torch.save(_sd(router_network), _path(filepath_models, "router_network", epoch))
    torch.save(_sd(router_optimizer), _path(filepath_models, "router_network_optim", epoch))


def save_training_state(filepath_models, epoch, moe, ema_helper=None):
    state = {"epoch": int(epoch), "step_count": _device_step(moe), "g_steps": list(moe.g_steps),
             "d_steps": list(moe.d_steps), "rng_counter": int(moe.rng.counter), "rng_seed": int(moe.rng_seed)}
    if ema_helper is not None:
        state["ema"] = ema_helper.state_dict()
    torch.save(state, _path(filepath_models, "train_state", epoch))


def _device_step(moe):
    return int(moe._dstep.item()) if getattr(moe, "_dstep", None) is not None else int(moe.step_count)


def save_checkpoint(filepath_models, epoch, moe, gen_optims, disc_optims, aux_reg_optims, router_optim,
                    ema_helper=None):
    save_models_and_architectures(filepath_models, moe.n_experts, moe.aux_regs, aux_reg_optims, moe.generators,
                                  gen_optims, moe.discriminators, disc_optims, moe.router, router_optim, epoch,
                                  multiple_aux_regs=True)
    save_training_state(filepath_models, epoch, moe, ema_helper)


def _load(path, device):
    return torch.load(path, map_location=device, weights_only=True)


def load_checkpoint_weights(checkpoint_dir, epoch, generators, generator_optimizers, discriminators,
                            discriminator_optimizers, aux_regs, aux_reg_optimizers, router_network, router_optimizer,
                            device="cuda"):
    """Restore every model and optimizer saved by save_models_and_architectures for ``epoch``."""
    groups = [("gen", generators, generator_optimizers), ("disc", discriminators, discriminator_optimizers),
              ("aux_reg", aux_regs, aux_reg_optimizers)]
    for name, mods, opts in groups:
        for i, m in enumerate(mods):
            m.load_state_dict(_load(_path(checkpoint_dir, name, epoch, i), device))
            if hasattr(m, "invalidate"):
                m.invalidate()
        for i, o in enumerate(opts):
            o.load_state_dict(_load(_path(checkpoint_dir, f"{name}_optim", epoch, i), device))
    router_network.load_state_dict(_load(_path(checkpoint_dir, "router_network", epoch), device))
    if hasattr(router_network, "invalidate"):
        router_network.invalidate()
    router_optimizer.load_state_dict(_load(_path(checkpoint_dir, "router_network_optim", epoch), device))


def load_checkpoint(checkpoint_dir, epoch, moe, gen_optims, disc_optims, aux_reg_optims, router_optim,
                    ema_helper=None, device="cuda"):
    """Models + optimizers + training state; the next train_step continues the saved run's streams."""
    load_checkpoint_weights(checkpoint_dir, epoch, moe.generators, gen_optims, moe.discriminators, disc_optims,
                            moe.aux_regs, aux_reg_optims, moe.router, router_optim, device)
    path = _path(checkpoint_dir, "train_state", epoch)
    if not os.path.exists(path):
        return None
    st = _load(path, "cpu")
    moe.step_count = int(st["step_count"])
    if getattr(moe, "_dstep", None) is not None:
        moe._dstep.fill_(moe.step_count)
    moe.g_steps, moe.d_steps = list(st["g_steps"]), list(st["d_steps"])
    moe.rng_seed = moe.rng.seed = int(st["rng_seed"])      # dropout / noise / Gumbel Philox key
    moe.rng.counter = int(st["rng_counter"])
    if ema_helper is not None and "ema" in st:
        ema_helper.load_state_dict(st["ema"])
    return st
