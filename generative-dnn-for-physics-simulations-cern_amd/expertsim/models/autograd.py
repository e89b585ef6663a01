"""torch.autograd bridges so the model classes keep the reference's nn.Module call API
(``G(noise, cond)``, ``D(img, cond)``, ``A(x)``) with ``loss.backward()`` working.

Forward/backward run the explicit HIP programs; parameter gradients are accumulated straight
into each module's flat gradient buffer (its ``p.grad`` views), which is where the fused Adam of
expertsim.optim reads them.  Gradients w.r.t. noise / cond are not produced (the reference never
needs them).  Dropout streams for module calls outside MoEWrapper.train_step come from a
per-module call counter, or — to replay a given run's masks, e.g. the reference goldens — from
``module.dropout_keys``, a list of (seed, stream_base) pairs consumed one per forward call
(stream_base = expertsim.utils.philox.dropout_stream(step, expert, pass, 0))."""
from __future__ import annotations

import torch

from ..layers import Act


def _img_tensor(act: Act):
    return act.torch_nchw()


def _dropout_key(module, pass_offset):
    keys = getattr(module, "dropout_keys", None)
    if keys:
        seed, base = keys.pop(0)
        return int(seed), int(base)
    module._calls = getattr(module, "_calls", 0) + 1
    return torch.initial_seed(), (1 << 30) + module._calls * 8 + pass_offset


class _GenFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, noise, cond, flat, module):
        seed, base = _dropout_key(module, 0)
        img, c = module.fwd(noise.contiguous().float(), cond.contiguous().float(), seed=seed, stream_base=base,
                            train=module.training)
        ctx.module, ctx.c = module, c
        return _img_tensor(img).clone()

    @staticmethod
    def backward(ctx, dimg):
        dimg = dimg.contiguous().float()
        ctx.module.bwd(ctx.c, Act.of(dimg))
        return None, None, None, None


class _DiscFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, cond, flat, module):
        out, lat, c = module.fwd(Act.of(img.contiguous().float()), cond.contiguous(), train=module.training)
        ctx.module, ctx.c = module, c
        ctx.need_img = img.requires_grad
        return out.rows2d().clone(), lat.rows2d().clone()

    @staticmethod
    def backward(ctx, dout, dlat):
        do = Act.of(dout.contiguous().float()) if dout is not None else None
        dl = Act.of(dlat.contiguous().float()) if dlat is not None else None
        dimg = ctx.module.bwd(ctx.c, do, dl, weight_grads=True, input_grad=ctx.need_img)
        return (dimg.torch_nchw().clone() if dimg is not None else None), None, None, None


class _AuxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, flat, module):
        seed, base = _dropout_key(module, 2)
        out, c = module.fwd(Act.of(img.contiguous().float()), seed=seed, stream_base=base, train=module.training)
        ctx.module, ctx.c = module, c
        ctx.need_img = img.requires_grad
        return out.rows2d().clone()

    @staticmethod
    def backward(ctx, dout):
        dimg = ctx.module.bwd(ctx.c, Act.of(dout.contiguous().float()), input_grad=ctx.need_img)
        return (dimg.torch_nchw().clone() if dimg is not None else None), None, None


def _anchor(module):
    # a tensor that requires grad so autograd records the node even for no-grad inputs
    flat = module.flat_params
    return flat.detach().requires_grad_(True)


def generator_apply(module, noise, cond):
    return _GenFn.apply(noise, cond, _anchor(module), module)


def discriminator_apply(module, img, cond):
    return _DiscFn.apply(img, cond, _anchor(module), module)


def aux_apply(module, img):
    return _AuxFn.apply(img, _anchor(module), module)
