"""Shared plumbing of the expertsim model classes.

* ``build_tree`` creates the reference's parameter tree (same dotted names, same construction
  order -> identical default init under the same torch seed, identical state_dict keys) from a
  declarative spec; layers without parameters (Dropout, LeakyReLU, Upsample, pools) are not
  materialised — their behaviour lives in each model's forward/backward program.
* ``ExpertModule.flatten`` moves every parameter into ONE contiguous fp32 buffer (and every
  gradient into one grad buffer) so the optimizer is a single fused Adam launch and the DDP
  all-reduce is a single bucket per model (see expertsim/train/training_setup.py).
"""
from __future__ import annotations

import torch
from torch import nn


def _container(root: nn.Module, path):
    mod = root
    for p in path:
        if p not in mod._modules:
            mod.add_module(p, nn.Module())
        mod = mod._modules[p]
    return mod


def build_tree(root: nn.Module, specs):
    """specs: list of (dotted_name, factory) in reference construction order."""
    for name, factory in specs:
        parts = name.split(".")
        parent = _container(root, parts[:-1])
        parent.add_module(parts[-1], factory())


def get_module(root: nn.Module, name: str) -> nn.Module:
    mod = root
    for p in name.split("."):
        mod = mod._modules[p]
    return mod


class ExpertModule(nn.Module):
    """Base of generator / discriminator / aux-regressor / router.

    Subclasses implement ``program(device)`` (build the HIP layer ops bound to the current
    parameter storage) and explicit ``fwd`` / ``bwd`` methods used by MoEWrapper.train_step."""

    compute_dtype = torch.float32

    def __init__(self):
        super().__init__()
        self._flat = None
        self._ops = None
        self._flat_ok = False      # flat storage verified since the last device move / reload
        self._offs = None

    # ----------------------------------------------------------------- flat parameter storage
    def flatten(self):
        if self._flat_ok and self._flat is not None:
            return
        params = [p for p in self.parameters()]
        dev = params[0].device
        total = sum(p.numel() for p in params)
        if self._flat is not None and self._flat[0].device == dev and self._flat[0].numel() == total \
                and all(p.data.data_ptr() == self._flat[0][o:o + p.numel()].data_ptr()
                        for p, o in zip(params, self._offsets())):
            self._flat_ok = True
            return
        flat_p = torch.empty(total, dtype=torch.float32, device=dev)
        flat_g = torch.zeros(total, dtype=torch.float32, device=dev)
        o = 0
        for p in params:
            n = p.numel()
            flat_p[o:o + n].copy_(p.data.reshape(-1))
            p.data = flat_p[o:o + n].view_as(p)
            p.grad = flat_g[o:o + n].view_as(p)
            o += n
        self._flat = (flat_p, flat_g)
        self._ops = None
        self._flat_ok = True

    def _offsets(self):
        if self._offs is None:
            o, out = 0, []
            for p in self.parameters():
                out.append(o)
                o += p.numel()
            self._offs = out
        return self._offs

    @property
    def flat_params(self):
        self.flatten()
        return self._flat[0]

    @property
    def flat_grads(self):
        self.flatten()
        return self._flat[1]

    def zero_grads(self):
        self.flatten()
        self._flat[1].zero_()
        g = self._flat[1]
        base = g.data_ptr()
        for p, o in zip(self.parameters(), self._offsets()):
            pg = p.grad
            # re-point only a gradient someone replaced (set_to_none elsewhere, autograd accumulate)
            if pg is None or pg.data_ptr() != base + 4 * o or pg.shape != p.shape:
                p.grad = g[o:o + p.numel()].view_as(p)

    def ops(self):
        """Layer ops bound to the flat parameter storage (rebuilt after device moves)."""
        self.flatten()
        if self._ops is None:
            self._ops = self.program()
            prefix = getattr(self, "_probe_prefix", None)
            for k, op in self._ops.items():
                if hasattr(op, "label"):
                    op.label = f"{prefix}.{k}" if prefix else None
        return self._ops

    def invalidate(self):
        """Called after every optimizer step: packed GEMM weights must be rebuilt.  The packings
        already made are rebuilt in place right here, batched (layers.repack_ops: one launch for the
        module instead of one or two per layout at its next use)."""
        if self._ops is not None:
            from ..layers import repack_ops
            repack_ops(self._ops.values())

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._flat = None
        self._ops = None
        self._flat_ok = False
        return out

    def _load_from_state_dict(self, *args, **kwargs):
        super()._load_from_state_dict(*args, **kwargs)
        self._flat_ok = False       # re-verify: loading copies in place, but a module may be rebuilt

    def __deepcopy__(self, memo):
        # deep copies (moe.py:29-31) must not share flat storage
        cls = self.__class__
        new = cls.__new__(cls)
        memo[id(self)] = new
        import copy as _copy
        for k, v in self.__dict__.items():
            if k in ("_flat", "_ops", "_offs"):
                setattr(new, k, None)
            elif k == "_flat_ok":
                setattr(new, k, False)
            else:
                setattr(new, k, _copy.deepcopy(v, memo))
        for p in new.parameters():
            p.grad = None
        return new
