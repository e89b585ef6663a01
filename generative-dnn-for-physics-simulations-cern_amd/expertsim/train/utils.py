"""Evaluation helpers — reference: expertsim/train/utils.py:18-205.

Same names, arguments and return conventions as the reference:
  get_channel_masks(a [H,W])                        train/utils.py:18-59   (host, numpy: geometry only)
  sum_channels_parallel(data [N,H,W])               train/utils.py:62-78   -> zip of 5-tuples
  get_max_value_image_coordinates(img)              train/utils.py:81-82
  calculate_joint_ws_across_experts(...)            train/utils.py:117-176
  get_predictions_from_generator_results(...)       train/utils.py:179-205

MI355X design: the generated images never leave the device.  Each generator batch is produced in
HBM (eval mode: BatchNorm running statistics, no dropout), and the fused HIP kernel
``es_channel_sums`` (csrc/eval.hip) applies expm1 and reduces every image to its five masked photon
sums in one pass, in fp64.  Only the [N,5] sums cross to the host, where the 1-D Wasserstein
distances are taken with scipy.stats.wasserstein_distance exactly as the reference does (a host
O(N log N) sort over a few thousand values per channel).  There is no CPU fallback for the sums:
``channel_sums`` raises when the HIP library or device is missing.
"""
from __future__ import annotations

import ctypes as C
from typing import List

import numpy as np
import torch

from .. import hip


def get_channel_masks(input_array: np.ndarray):
    """Masks 1..5 of train/utils.py:18-59 for an [n, m] image: mask5 = the squares with (i+j) even;
    masks 1..4 split the (i+j)-odd squares into the bottom-left, bottom-right, top-left and
    top-right quadrants (split at n//2, m//2)."""
    n, m = np.asarray(input_array).shape
    i = np.arange(n)[:, None]
    j = np.arange(m)[None, :]
    odd = ((i + j) & 1).astype(np.float64)
    top = (i < n // 2)
    left = (j < m // 2)
    dt = np.asarray(input_array).dtype
    mask1 = (odd * (~top & left)).astype(dt)
    mask2 = (odd * (~top & ~left)).astype(dt)
    mask3 = (odd * (top & left)).astype(dt)
    mask4 = (odd * (top & ~left)).astype(dt)
    mask5 = (1.0 - odd).astype(dt)
    return mask1, mask2, mask3, mask4, mask5


def _as_device_images(data, device=None) -> torch.Tensor:
    t = data if isinstance(data, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(data))
    if t.dim() == 4:
        if t.shape[1] != 1:
            raise ValueError(f"channel sums need one-channel images, got {tuple(t.shape)}")
        t = t[:, 0]
    if t.dim() != 3:
        raise ValueError(f"channel sums need images [N,H,W], got {tuple(t.shape)}")
    if t.dtype not in (torch.float32, torch.bfloat16):
        t = t.float()
    if not t.is_cuda:
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        t = t.to(dev, non_blocking=True)
    return t


def channel_sums(images, log_domain: bool = False, device=None) -> torch.Tensor:
    """[N,5] fp64 device tensor of the five masked sums of each image (HIP kernel es_channel_sums).

    images: [N,H,W] or [N,1,H,W], fp32 / bf16, any strides, device or host (host data is copied
    to the device first).  log_domain=True sums expm1(images) (the log1p-domain images of the
    dataset and generator, moe.py:646, train/utils.py:198), fused into the same pass."""
    x = _as_device_images(images, device)
    N, H, W = x.shape
    out = torch.empty(N, 5, dtype=torch.float64, device=x.device)
    if N == 0:
        return out
    view = hip.make_view((N, 1, H, W), (x.stride(0), H * W, x.stride(1), x.stride(2)))
    with torch.cuda.device(x.device):
        hip.call("es_channel_sums", C.byref(view), hip.dt_of(x), C.c_void_p(x.data_ptr()),
                 1 if log_domain else 0, hip.ptr(out), hip.stream_ptr())
    return out


def sum_channels_parallel(data):
    """Reference API (train/utils.py:62-78): zip of (ch1, ch2, ch3, ch4, ch5) per image."""
    s = channel_sums(data).cpu().numpy()
    return zip(s[:, 0], s[:, 1], s[:, 2], s[:, 3], s[:, 4])


def get_max_value_image_coordinates(img):
    """train/utils.py:81-82 (host helper used by the data pipeline)."""
    return np.unravel_index(np.argmax(img), img.shape)


def _generate_log_images(generator, noise: torch.Tensor, cond: torch.Tensor) -> torch.Tensor:
    """One eval-mode generator batch -> log1p-domain images [n,H,W] on the device."""
    generator.eval()                 # the reference leaves the generator in eval mode (utils.py:195)
    if hasattr(generator, "fwd"):    # expertsim HIP generator: skip the autograd bridge's copy
        img, _ = generator.fwd(noise.contiguous(), cond.contiguous(), train=False)
        t = img.torch_nchw()
    else:
        t = generator(noise, cond)
    t = t.reshape(t.shape[0], -1, t.shape[-2], t.shape[-1])
    return t[:, 0]


def _cond_on(y, device):
    y = y if isinstance(y, torch.Tensor) else torch.as_tensor(np.asarray(y))
    return y.to(device=device, dtype=torch.float32)


@torch.no_grad()
def generator_channel_sums(batch_size, num_samples, noise_dim, device, y_test, generator,
                           input_noise=None) -> torch.Tensor:
    """Device-resident core of get_predictions_from_generator_results + sum_channels_parallel:
    [num_samples, 5] fp64 sums of expm1(G(noise, cond)), batch by batch, images never copied out."""
    out = torch.empty(num_samples, 5, dtype=torch.float64, device=device)
    y = _cond_on(y_test, device)
    for start in range(0, num_samples, batch_size):
        end = min(start + batch_size, num_samples)
        if input_noise is not None:
            noise = _cond_on(input_noise[start:end], device)
        else:
            noise = torch.randn(end - start, noise_dim, device=device)
        imgs = _generate_log_images(generator, noise, y[start:end])
        out[start:end] = channel_sums(imgs, log_domain=True)
    return out


@torch.no_grad()
def get_predictions_from_generator_results(batch_size, num_samples, noise_dim, device, y_test, generator,
                                           shape_images=(56, 30), input_noise=None):
    """Reference API (train/utils.py:179-205): host arrays (expm1(images), images), float64."""
    res = np.zeros((num_samples, *shape_images))
    raw = np.zeros((num_samples, *shape_images))
    y = _cond_on(y_test, device)
    for start in range(0, num_samples, batch_size):
        end = min(start + batch_size, num_samples)
        if input_noise is not None:
            noise = _cond_on(input_noise[start:end], device)
        else:
            noise = torch.randn(end - start, noise_dim, device=device)
        r = _generate_log_images(generator, noise, y[start:end]).float().cpu().numpy()
        res[start:end] = np.expm1(r).reshape(-1, *shape_images)
        raw[start:end] = r.reshape(-1, *shape_images)
    return res, raw


def calculate_joint_ws_across_experts(n_calc, x_tests: List, y_tests: List, generators: List, ch_org,
                                      ch_org_expert, noise_dim, device, batch_size=64, n_experts=3,
                                      shape_images=(56, 30)):
    """Reference API and arithmetic (train/utils.py:117-176): for each of n_calc repetitions,
    generate every expert's samples, take the 5-channel WS distance of the joint and of each
    expert's distribution against the real sums, average over channels, then mean/std over the
    repetitions.  Returns (ws_mean, ws_std, ws_mean_exp [E], ws_std_exp [E])."""
    from scipy.stats import wasserstein_distance
    if len(x_tests) != len(y_tests) or len(x_tests) != len(generators):
        raise ValueError("Length of data is not the same")
    ch_org = np.asarray(ch_org)
    ws = np.zeros((n_calc, 5))
    ws_exp = np.zeros((n_calc, n_experts, 5))
    for j in range(n_calc):
        per = []
        for g_idx, gen in enumerate(generators):
            num = int(np.asarray(x_tests[g_idx]).shape[0]) if not isinstance(x_tests[g_idx], torch.Tensor) \
                else int(x_tests[g_idx].shape[0])
            if num == 0:
                per.append(None)
                continue
            per.append(generator_channel_sums(batch_size, num, noise_dim, device, y_tests[g_idx], gen))
        live = [p for p in per if p is not None]
        ch_gen_all = torch.cat(live).cpu().numpy() if live else np.zeros((0, 5))
        ch_gen_exp = [p.cpu().numpy() if p is not None else np.array([]) for p in per]
        for i in range(5):
            ws[j][i] = wasserstein_distance(ch_org[:, i], ch_gen_all[:, i])
            for e in range(len(generators)):
                org_e = np.asarray(ch_org_expert[e])
                if ch_gen_exp[e].shape[0] == 0 or org_e.shape[0] == 0:
                    continue
                ws_exp[j][e][i] = wasserstein_distance(org_e[:, i], ch_gen_exp[e][:, i])
    ws_runs = ws.mean(axis=1)
    ws_exp_runs = ws_exp.mean(axis=2)
    return ws_runs.mean(), ws_runs.std(), ws_exp_runs.mean(axis=0), ws_exp_runs.std(axis=0)
