"""Diagnostic: proton generator backward, layer by layer (activation gradients), HIP vs torch fp32.

usage: python tools/diag_gbwd_layers.py <B>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import bench  # noqa: E402
from expertsim import hip  # noqa: E402
from expertsim.layers import Act, act_bwd  # noqa: E402
from oracle import expertsim_oracle as O  # noqa: E402

B = int(sys.argv[1])
moe, opts, cfg = bench.build("proton", 1, "fp32", 1234, torch.device("cuda"))
G = moe.generators[0]
gen = torch.Generator().manual_seed(B)
noise, cond = torch.randn(B, 10, generator=gen), torch.randn(B, 9, generator=gen)
dimg = torch.randn(B, 1, 56, 30, generator=gen)
G.zero_grads()
img, c = G.fwd(noise.cuda(), cond.cuda(), seed=1234, stream_base=0, train=True)
o = G.ops()
lr = hip.chain_struct(hip.ACT_LRELU, 0.1)
g = lambda n, a="weight": getattr(G.get_submodule(n), a).grad
rec = {}
dh6 = act_bwd(c["h6"], hip.chain_struct(hip.ACT_RELU), Act.of(dimg.cuda().contiguous()), dx_dtype=torch.float32)
rec["dh6"] = dh6
dy5 = o["c11"].dgrad(dh6, c["y5"]); rec["dy5"] = dy5
dh5 = o["gn3"].bwd(c["h5"], c["s5"], lr, dy5, dgamma=g("conv_layers.9"), dbeta=g("conv_layers.9", "bias"),
                   dsum=g("conv_layers.8", "bias")); rec["dh5"] = dh5
dy4 = o["c8"].dgrad(dh5, c["y4"]); rec["dy4"] = dy4
dh4 = o["gn2"].bwd(c["h4"], c["s4"], lr, dy4, dgamma=g("conv_layers.6"), dbeta=g("conv_layers.6", "bias"),
                   dsum=g("conv_layers.5", "bias")); rec["dh4"] = dh4
dy3 = o["c5"].dgrad(dh4, c["y3"]); rec["dy3"] = dy3
dh3 = o["gn1"].bwd(c["h3"], c["s3"], lr, dy3, dgamma=g("conv_layers.2"), dbeta=g("conv_layers.2", "bias"),
                   dsum=g("conv_layers.1", "bias")); rec["dh3"] = dh3
torch.cuda.synchronize()

P = O.build_all("proton", 1, 1234)["G"][0]
T = {}
x = torch.cat((noise, cond), 1)
ln = lambda t, n, shape: F.layer_norm(t, shape, P[f"{n}.weight"], P[f"{n}.bias"], 1e-5)
gn = lambda t, n: F.group_norm(t, 32, P[f"{n}.weight"], P[f"{n}.bias"], 1e-5)
lrelu = lambda t: F.leaky_relu(t, 0.1)
keep = lambda name, t: (t.retain_grad(), T.__setitem__(name, t), t)[2]
x = lrelu(ln(O._lin(x, P, "fc1.0"), "fc1.1", (256,)))
x = lrelu(ln(O._lin(x, P, "fc2.0"), "fc2.1", (512 * 18 * 10,)))
x = x.view(-1, 512, 18, 10).detach().requires_grad_(True)
x2 = F.interpolate(x, scale_factor=(2, 2), mode="nearest")
h3 = keep("dh3", O._conv(x2, P, "conv_layers.1", padding=1))
y3 = keep("dy3", lrelu(gn(h3, "conv_layers.2")))
x3 = F.interpolate(y3, size=(56, 30), mode="nearest")
h4 = keep("dh4", O._conv(x3, P, "conv_layers.5", padding=1))
y4 = keep("dy4", lrelu(gn(h4, "conv_layers.6")))
h5 = keep("dh5", O._conv(y4, P, "conv_layers.8", padding=1))
y5 = keep("dy5", lrelu(gn(h5, "conv_layers.9")))
h6 = keep("dh6", O._conv(y5, P, "conv_layers.11", padding=1))
out = F.relu(h6)
(out * dimg).sum().backward()
print(f"B={B} image err {float((img.torch_nchw().cpu() - out.detach()).abs().max()):.2e}")
for k in ("dh6", "dy5", "dh5", "dy4", "dh4", "dy3", "dh3"):
    mine = rec[k].torch_nchw().float().cpu()
    ref = T[k].grad
    print(f"  {k}: shape {tuple(ref.shape)} normrel {float((mine - ref).norm() / ref.norm()):.2e}  "
          f"maxabs {float((mine - ref).abs().max()):.2e} |ref|max {float(ref.abs().max()):.2e}")

# --- the GN backward of layer gn3 again: on the generator's own Acts vs dense copies
from expertsim.layers import Act as _A  # noqa: E402
print("h5 view", c["h5"].dims, c["h5"].strides, c["h5"].t.dtype, tuple(c["h5"].t.shape),
      "| dy5 view", dy5.dims, dy5.strides, tuple(dy5.t.shape))
def dense(a):
    t = a.torch_nchw().float().contiguous(memory_format=torch.channels_last)
    return _A(t, tuple(t.shape), tuple(t.stride()))
for label, (xx, dd) in {"own": (c["h5"], dy5), "dense": (dense(c["h5"]), dense(dy5))}.items():
    dxx = o["gn3"].bwd(xx, c["s5"], lr, dd)
    torch.cuda.synchronize()
    mine = dxx.torch_nchw().float().cpu()
    print(f"  gn3 bwd on {label}: normrel vs torch {float((mine - T['dh5'].grad).norm() / T['dh5'].grad.norm()):.2e}")

# --- float64 truth of the gn3 backward on the HIP forward's own h5
h5d = c["h5"].torch_nchw().double().cpu().requires_grad_(True)
P9w, P9b = P["conv_layers.9.weight"].double(), P["conv_layers.9.bias"].double()
z = F.group_norm(h5d, 32, P9w, P9b, 1e-5)
F.leaky_relu(z, 0.1).backward(dy5.torch_nchw().double().cpu())
truth = h5d.grad
mine = rec["dh5"].torch_nchw().double().cpu()
print(f"  truth(fp64 on HIP h5) vs HIP {float((mine - truth).norm() / truth.norm()):.2e}, "
      f"vs torch-fp32 path {float((T['dh5'].grad.double() - truth).norm() / truth.norm()):.2e}")
err = (mine - truth).reshape(B, 32, -1).norm(dim=2) / truth.reshape(B, 32, -1).norm(dim=2)
print("  per-(n, group) rel err > 1e-4:", [(int(i), int(j), float(err[i, j])) for i, j in (err > 1e-4).nonzero()][:20])
zz = z.detach().reshape(B, 32, -1)
print("  |z| < 1e-4 count:", int((zz.abs() < 1e-4).sum()), "of", zz.numel())
