"""The BASELINE.json GPU workloads through the HIP path, in the fp32 parity mode (the bench headline
since round 3) and the bf16 performance mode, checked by size-independent properties (the elementwise parity pins are the fp32 goldens in
test_train_step_gpu.py / test_grads_gpu.py; bf16 statistical parity is test_bf16_stats_gpu.py):

  configs[1]  neutron 44x44, E=1, B=512
  configs[2]  neutron 44x44, E=1, B=1024 (the bench headline)
  configs[3]  neutron 44x44, E=4, B=512 per GPU (the per-rank shard of the 4-GPU B=2048 run)
  configs[4]  neutron56 56x56 (declared extension, parity unpinned), E=8, B=512 per GPU
  + proton 56x30, E=1, B=512 (the reference's other model family)

Each runs 3 train steps: every metric is finite and the metric-key set is the reference's
(moe.py:480-502); per-expert counts sum to B; generated images are >= 0 (ReLU output) and the
parameters of every model moved; with E=1 the step also captures and replays as a HIP graph at
this batch (finite metrics, parameters move; replay == eager is test_graph_gpu.py).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

CONFIGS = [("neutron", 1, 512), ("neutron", 1, 1024), ("neutron", 4, 512), ("neutron56", 8, 512),
           ("proton", 1, 512)]


def _keys(E):
    k = {"gen_loss", "disc_loss", "div_loss", "intensity_loss", "aux_reg_loss", "router_loss",
         "expert_distribution_loss", "differentiation_loss", "expert_entropy_loss",
         "adaptive_load_balancing_loss", "gan_loss"}
    for i in range(E):
        k |= {f"gen_loss_{i}", f"disc_loss_{i}", f"div_loss_experts_{i}", f"intensity_loss_experts_{i}",
              f"aux_reg_loss_experts_{i}", f"std_intensities_experts_{i}", f"mean_intensities_experts_{i}",
              f"n_choosen_experts_mean_epoch_{i}"}
    return k


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("arch,E,B", CONFIGS)
def test_config_steps(arch, E, B, precision):
    import bench
    from expertsim.utils.synthetic import make_batch
    moe, (og, od, oa, orr), cfg = bench.build(arch, E, precision, 1234, torch.device(DEV))
    b = make_batch(B, arch, seed=5)
    t = {k: torch.from_numpy(v).to(DEV) for k, v in b.items()}
    real = t["real_images"].unsqueeze(1).contiguous()
    args = (0, t["cond"], real, t["true_positions"], t["std"], t["intensity"], oa, og, od, orr, None, DEV)
    p0 = {n: p.detach().clone() for n, p in moe.named_parameters()}
    for s in range(3):
        m = moe.train_step(*args)
        torch.cuda.synchronize()
        mf = {k: float(v) for k, v in m.items()}
        assert set(mf) == _keys(E)
        bad = [k for k, v in mf.items() if not math.isfinite(v)]
        assert not bad, (s, bad)
        assert sum(mf[f"n_choosen_experts_mean_epoch_{i}"] for i in range(E)) == B
    moved = {n for n, p in moe.named_parameters() if not torch.equal(p.detach(), p0[n])}
    for pref in ("generators", "discriminators", "aux_regs"):
        assert any(n.startswith(pref) for n in moved), pref
    # eval-mode generator output of the trained model is a valid image batch
    with torch.no_grad():
        img, _ = moe.generators[0].fwd(t["cond"].new_zeros(8, 10).normal_(), t["cond"][:8], train=False)
        x = img.torch_nchw()
    assert x.shape == (8, 1, *moe.image_shape) and bool(torch.isfinite(x).all()) and float(x.min()) >= 0.0
    if E == 1:
        from expertsim.graph import StepGraph
        sg = StepGraph(moe, args, warmup=1)
        torch.cuda.synchronize()
        state = {n: p.detach().clone() for n, p in moe.named_parameters()}
        mg = {k: float(v) for k, v in sg.replay().items()}
        torch.cuda.synchronize()
        assert all(math.isfinite(v) for v in mg.values())
        assert any(not torch.equal(p.detach(), state[n]) for n, p in moe.named_parameters())
