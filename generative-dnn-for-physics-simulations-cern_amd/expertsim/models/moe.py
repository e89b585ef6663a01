"""MoEWrapper — the expertsim GAN training step on MI355X.

Reference: expertsim/models/moe.py:14-699 (``MoEWrapper.__init__`` 24-50, ``train_step`` 52-504,
``discriminator_train_step`` 506-527, ``generator_train_step`` 529-571,
``sdi_gan_regularization`` 573-588, ``intensity_regularization`` 590-642).

Same constructor and ``train_step`` signature and the same metric keys (moe.py:480-502).  The step
is an explicit program of HIP kernels (no autograd): router -> per expert {G fwd #1, D step
(D(real), D(fake), hinge, D backward, fused Adam), G fwd #2, D(fake1), D(fake2), aux regressor,
fused G losses, D/A/G backward, fused Adam} -> router loss + Adam.  Loss weights and metrics stay
on the device and nothing synchronises with the host.

Multi-expert steps (n_experts > 1) run on DYNAMIC ROWS: every expert's program is issued on buffers
of the batch's capacity B with the expert's sample count read on the device (es_expert_plan:
live rows, the reference's ``B_e <= 1`` skip rule of moe.py:126 as an ``active`` flag gating the
expert's Adam / spectral-norm / batch-counter updates, loss weights, data-parallel offsets), so the
step's launches do not depend on the routing: no host round trip, and single-process steps replay
as one captured HIP graph per expert whatever the expert sizes (hip.live_rows).

Randomness: noise / Gumbel draws come from device Philox streams unless ``noise_fn`` /
``gumbel_fn`` inject them (parity tests); dropout masks are Philox streams keyed by
(step, expert, pass, layer) at the GLOBAL element index (data-parallel ranks draw their rows of the
single-device draws) — expertsim/utils/philox.py.

Data parallel (expertsim/train/ddp.py): with ``self.ddp`` set, each rank routes its own shard,
gradients of every optimizer phase are all-reduced (RCCL) before the fused Adam; with
``ddp.sync_bn`` the batch-coupled statistics are global and the step equals the single-device
step of the global batch.
"""
from __future__ import annotations


import contextlib
import copy
import ctypes as C

import numpy as np
import torch
from torch import nn

from .. import hip
from ..config import cfg_get
from ..layers import (Act, batch_live_counts, copy_act, defer_num_batches, set_deterministic, set_f32_split,
                      set_norm_sync)
from ..rng import DeviceRNG
from ..utils import philox


class MoEWrapper(nn.Module):
    name = "separate-gumbal-gen-disc-shared-aux-reg-masked-router-multiple-aux-reg"
    description = "MoEWrapper where expert is defined as a generator and discriminator." \
                  "Auxiliary regressor is each for every expert "

    def __init__(self, generator_cls, discriminator_cls, aux_reg_cls, router_cls, n_experts: int, cfg,
                 image_shape: tuple = (56, 30)):
        super().__init__()
        self.image_shape = tuple(image_shape)
        self.generators = nn.ModuleList([copy.deepcopy(generator_cls) for _ in range(n_experts)])
        self.discriminators = nn.ModuleList([copy.deepcopy(discriminator_cls) for _ in range(n_experts)])
        self.aux_regs = nn.ModuleList([copy.deepcopy(aux_reg_cls) for _ in range(n_experts)])
        self.router = router_cls
        self.n_experts = n_experts
        for i in range(n_experts):
            self.generators[i]._probe_prefix = f"G{i}"
            self.discriminators[i]._probe_prefix = f"D{i}"
            self.aux_regs[i]._probe_prefix = f"A{i}"
        self.noise_dim = int(cfg.model.noise_dim)
        self.cfg = cfg
        self.g_steps = [0 for _ in range(n_experts)]
        self.d_steps = [0 for _ in range(n_experts)]
        self.rng_seed = int(cfg_get(cfg, "train.rng_seed", 1234))
        self.rank = 0
        self.rng = DeviceRNG(self.rng_seed)
        self.noise_fn = None       # optional injection: fn(expert, which, shape) -> tensor
        self.gumbel_fn = None      # optional injection: fn(shape) -> Exp(1) tensor
        self.ddp = None            # expertsim.train.ddp.DataParallel (set by the loop)
        self.step_count = 0
        self._ed_feat = None       # [B] per-sample photon sums for the router's ED term
        self._w_cache = {}         # class_counts_adjusted device scalars
        self.expert_graphs = bool(cfg_get(cfg, "train.expert_graphs", True))
        self.expert_graphs_concurrent = True
        self._egraphs = None       # ExpertGraphs (n_experts > 1, single process)
        self._graphs = None
        self._static = None
        self._bufs = {}
        self._eager_steps = 0
        self._expert_eager = set()  # experts that have run one eager step (then graph-capturable)
        self._dstep = None         # device int32 step counter: dropout / noise streams (graph replay)
        # fp32 parity mode: every float reduction in a fixed order (bitwise-reproducible steps)
        self.deterministic = bool(cfg_get(cfg, "train.deterministic", True))
        # fp32 conv arithmetic: "exact" (v_mfma_f32_16x16x4_f32) or "split" (three bf16 planes per
        # operand, six plane products on the bf16 MFMA; es_conv_set_f32_split)
        self.fp32_mfma = str(cfg_get(cfg, "train.fp32_mfma", "split"))
        if self.fp32_mfma not in ("exact", "split"):
            raise ValueError(f"train.fp32_mfma must be exact or split, got {self.fp32_mfma!r}")
        self.set_precision(cfg_get(cfg, "train.precision", "fp32"))

    def set_precision(self, precision: str):
        """fp32: every GEMM on fp32 MFMA (parity mode).  bf16: generator and aux-regressor GEMM
        operands and activations in bf16 (fp32 accumulation, statistics, parameters, optimizer);
        the discriminator stays fp32."""
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be fp32 or bf16, got {precision!r}")
        self.precision = precision
        low = torch.bfloat16 if precision == "bf16" else torch.float32
        for m in self.generators:
            m.compute_dtype = low
        for m in self.aux_regs:
            m.compute_dtype = low
        for m in self.discriminators:
            m.compute_dtype = torch.float32

    # ---------------------------------------------------------------------------- helpers
    # stream indices of the step's draws: Gumbel 0, expert e's noise_1 / noise_2 1 + 2e / 2 + 2e
    # (fixed per call site: a captured per-expert graph draws the same streams in every step)
    def _noise(self, expert, which, shape, device, row0=0):
        """row0: the rows' first index in the expert's global batch (data parallel); a device int32 [1]
        under dynamic rows (es_expert_plan n0)."""
        if self.noise_fn is not None:
            try:
                z = self.noise_fn(expert, which, shape)
            except KeyError:      # injected draws of the reference's active experts only: an expert
                z = torch.zeros(0, *shape[1:])   # it skipped runs on zero live rows here
            z = z.to(device=device, dtype=torch.float32)
            if z.shape[0] < shape[0]:    # dynamic rows: the injected draw covers the live rows only
                z = torch.cat([z, torch.zeros(shape[0] - z.shape[0], *shape[1:], dtype=z.dtype, device=device)])
            return z.contiguous()
        out = torch.empty(shape, dtype=torch.float32, device=device)
        if isinstance(row0, torch.Tensor):
            return self.rng.normal_at(out, 1 + 2 * expert + which, off_ptr=row0, off_mul=shape[1])
        return self.rng.normal_at(out, 1 + 2 * expert + which, offset=row0 * shape[1])

    def _gumbel(self, shape, device, row0=0):
        if self.gumbel_fn is not None:
            return self.gumbel_fn(shape).to(device=device, dtype=torch.float32).contiguous()
        return self.rng.exponential_at(torch.empty(shape, dtype=torch.float32, device=device), 0,
                                       offset=row0 * shape[1])

    def _expert_graphs_on(self, E):
        """Per-expert graph replay: multi-expert, single process, device randomness, and after one
        eager step (optimizer moments, packed weights and step counters exist outside any graph)."""
        return (self.expert_graphs and E > 1 and self.ddp is None and self.noise_fn is None
                and self.gumbel_fn is None and self._eager_steps >= 1 and not torch.cuda.is_current_stream_capturing())

    def _weight_scalar(self, be, B, dev):
        """class_counts_adjusted as a device scalar, one per distinct value (created outside any
        graph capture, no fill launch per step)."""
        w = float(np.float32(be) / np.float32(B))
        t = self._w_cache.get((w, dev))
        if t is None:
            t = self._w_cache[(w, dev)] = torch.full((1,), w, dtype=torch.float32, device=dev)
        return t

    def _buf(self, name, shape, dtype, dev):
        """A persistent device buffer (same storage every step)."""
        t = self._bufs.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.device != dev or t.dtype != dtype:
            t = self._bufs[name] = torch.empty(shape, dtype=dtype, device=dev)
            if self._egraphs is not None:
                self._egraphs.clear()        # graphs captured against the old buffer
        return t

    def _static_inputs(self, dev, *ts):
        shapes = tuple(tuple(t.shape) for t in ts)
        if self._static is None or self._static[0] != shapes:
            self._static = (shapes, [torch.empty_like(t) for t in ts])
            if self._egraphs is not None:
                self._egraphs.clear()
        out = self._static[1]
        for d, t in zip(out, ts):
            if d.data_ptr() != t.data_ptr():
                d.copy_(t)
        return out

    def _allreduce(self, module, average=True):
        if self.ddp is not None:
            self.ddp.allreduce_grads(module, average)

    # ---------------------------------------------------------------------------- the step
    def train_step(self, epoch, cond, real_images, true_positions, std, intensity, aux_reg_optimizers,
                   generator_optimizers, discriminator_optimizers, router_optimizer, ema_helper, device):
        dev = torch.device(device) if not isinstance(device, torch.device) else device
        if dev.type != "cuda":
            raise hip.HipError("MoEWrapper.train_step runs on the HIP device only (no CPU fallback)")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        E = self.n_experts
        f32 = lambda t: t.to(device=dev, dtype=torch.float32).contiguous()
        cond, real_images, true_positions, std, intensity = map(f32, (cond, real_images, true_positions,
                                                                     std, intensity))
        if real_images.dim() == 3:
            real_images = real_images.unsqueeze(1)
        B = cond.shape[0]
        step = self.step_count
        self._graphs = None
        if self._expert_graphs_on(E):
            # per-expert HIP graphs (ExpertGraphs): the batch lives in static buffers the graphs read
            cond, real_images, true_positions, std, intensity = self._static_inputs(
                dev, cond, real_images, true_positions, std, intensity)
            conc = self._experts_concurrent(E, B)
            if self._egraphs is None or self._egraphs.concurrent != conc:
                self._egraphs = ExpertGraphs(concurrent=conc)
            self._graphs = self._egraphs
        rc = self.cfg.model.router
        if self._dstep is None or self._dstep.device != dev:
            self._dstep = torch.full((1,), step, dtype=torch.int32, device=dev)
        # every step-dependent random stream is keyed on the device counter (captured graphs)
        hip.set_step_counter(self._dstep)
        self.rng.begin_step(self._dstep)
        set_deterministic(self.precision == "fp32" and self.deterministic)
        set_f32_split(self.fp32_mfma == "split")
        try:
            with defer_num_batches():
                return self._train_step(epoch, cond, real_images, true_positions, std, intensity,
                                        aux_reg_optimizers, generator_optimizers, discriminator_optimizers,
                                        router_optimizer, dev, B)
        finally:
            hip.set_step_counter(None)
            self.rng.end_step()

    def _train_step(self, epoch, cond, real_images, true_positions, std, intensity, aux_reg_optimizers,
                    generator_optimizers, discriminator_optimizers, router_optimizer, dev, B):
        E = self.n_experts
        step = self.step_count
        rc = self.cfg.model.router

        ddp = self.ddp
        tau = max(rc.tau_min, rc.tau_start * (rc.tau_decay ** epoch))          # moe.py:62-74
        expo = self._gumbel((B, E), dev, row0=(ddp.rank * B if ddp is not None else 0))
        gates, logits, idx, counts, rctx = self.router.fwd(cond, expo, tau)

        for i in range(E):                                                       # moe.py:115-119
            aux_reg_optimizers[i].zero_grad(set_to_none=True)
            generator_optimizers[i].zero_grad(set_to_none=True)
            discriminator_optimizers[i].zero_grad(set_to_none=True)
        router_optimizer.zero_grad(set_to_none=True)

        # expert dispatch (moe.py:97-99,121-123): E == 1 needs no routing at all; otherwise the
        # rows are grouped per expert on the device (es_router_dispatch) and the per-expert plan
        # (live rows, skip rule, loss weights, data-parallel offsets) is computed on the device
        plan = None
        if E == 1:
            groups = [(0, None, B)]
            if ddp is not None:
                groups = ddp.global_groups(groups, B)
        else:
            perm = self._buf("perm", (B,), torch.int32, dev)
            offs = self._buf("offs", (E + 1,), torch.int32, dev)
            hip.call("es_router_dispatch", hip.ptr(idx), B, E, hip.ptr(perm), hip.ptr(offs), hip.stream_ptr())
            plan = self._plan(counts, B, dev)
            groups = [(e, (perm, offs), B) for e in range(E)]

        # metrics buffer: per expert [total, gen, div, int, aux, std_int, mean_int, w, disc]
        # (persistent buffers: captured expert graphs write into them)
        mbuf = self._buf("mbuf", (E, 9), torch.float32, dev).zero_()
        # mean_intensities_in_batch_expert (moe.py:196-198): the ED router term's per-sample features
        self._ed_feat = (self._buf("ed_feat", (B,), torch.float32, dev).zero_()
                         if E > 1 and float(rc.ed_strength) != 0.0 else None)
        if self._graphs is not None:
            self._graphs.begin()
        # several experts: their programs fork onto their own streams (no shared parameters, disjoint
        # rows of the step's buffers), joined back before the router -- inside a whole-step capture
        # of one process (graph.StepGraph), and in eager data-parallel steps, where each expert's
        # collectives run on a communicator of its own (ddp.expert_groups).  (Eager single-process
        # steps replay the experts' own graphs concurrently instead, ExpertGraphs.)  A captured
        # data-parallel step runs its experts one after another: torch's ProcessGroupNCCL aborts when
        # collectives are issued from forked streams inside a capture (measured: its watchdog queried
        # an event recorded in the capture, "operation not permitted on an event last recorded in a
        # capturing stream"; a segmentation fault with its event cache off; tools/ddp_e4_probe.py)
        fork = None
        capturing = torch.cuda.is_current_stream_capturing()
        if plan is not None and self._experts_concurrent(E, B) and capturing == (ddp is None):
            if ddp is not None:
                ddp.ensure_expert_groups(E)
            fork = self._fork_streams(E)
        for e, rows, be in groups:
            og, od, oa = generator_optimizers[e], discriminator_optimizers[e], aux_reg_optimizers[e]
            if plan is not None:
                # dynamic rows: every expert's program is issued (B-sample capacity, live count and
                # the B_e <= 1 skip rule read on the device), so one graph per expert serves every step
                run = lambda e=e, rows=rows, og=og, od=od, oa=oa: self._expert_step(
                    e, rows, B, B, cond, real_images, true_positions, std, intensity, og, od, oa, mbuf, step, dev,
                    plan)
                if fork is not None:
                    with torch.cuda.stream(fork[e]):
                        run()
                elif self._graphs is not None and e in self._expert_eager:
                    for o in (og, od, oa):
                        o.prepare()      # (no lazy state creation inside a capture)
                    self._graphs.run((e, B), run)
                else:
                    run()
                    self._expert_eager.add(e)
                continue
            be_global = be if ddp is None else ddp.global_count(e)
            if be_global <= 1:                                                   # moe.py:126-135
                continue
            # SyncBN: global batch statistics, so even one local sample runs
            if be > 1 or (ddp is not None and ddp.sync_bn and be >= 1):
                run = lambda: self._expert_step(e, rows, be, B, cond, real_images, true_positions, std, intensity,
                                                og, od, oa, mbuf, step, dev)
                if self._graphs is not None and e in self._expert_eager:
                    self._weight_scalar(be, B, dev)
                    for o in (og, od, oa):
                        o.prepare()      # (no lazy state creation inside a capture)
                    self._graphs.run((e, be, B), run)
                else:
                    # an expert's first step runs eagerly (its optimizer moments, step counters and
                    # scratch then exist outside any graph), also when it first trains after step 0
                    run()
                    self._expert_eager.add(e)
            else:
                # DDP: expert active globally but (almost) absent from this shard -> zero local
                # gradients, but join the same collectives (same ranges, same order: D, A, then G's
                # backward buckets) and optimizer steps as the other ranks
                G_, D_, A_ = self.generators[e], self.discriminators[e], self.aux_regs[e]
                ddp.allreduce_async(D_)
                ddp.wait_all()
                od.step()
                ddp.allreduce_async(A_)
                ready = ddp.bucketer(G_)
                for name in G_.READY:
                    ready(name)
                ddp.wait_all()
                og.step()
                oa.step()

        if self._graphs is not None:
            self._graphs.join()
        if fork is not None:
            cur = torch.cuda.current_stream()
            for st in set(fork):
                cur.wait_stream(st)
        if ddp is not None:
            # the global batch's per-expert metrics on every rank
            ddp.merge_metrics(mbuf, None if plan is None else plan["lcnt"])

        # ---- router (moe.py:213-449)
        rl = None
        flags, dec_w = 0, 1.0
        if E > 1:
            alpha = min(max(epoch / rc.alpha, 0.0), 1.0)
            dec_w = rc.min_weight + (1.0 - rc.min_weight) * alpha
            # ALB, utilisation entropy and expert-distribution terms + d/dlogits in one program
            rl = torch.zeros(3, dtype=torch.float32, device=dev)
            dlogits = torch.empty(B, E, dtype=torch.float32, device=dev)
            ed_on = float(rc.ed_strength) != 0.0
            colsum = feat_all = idx_all = None
            B_tot, B_all = B, B
            if ddp is not None:
                # the ALB / entropy terms see the global gate sums, the ED term the global batch
                colsum = torch.empty(E, dtype=torch.float32, device=dev)
                hip.call("es_router_colsum", hip.ptr(gates), B, E, hip.ptr(colsum), hip.stream_ptr())
                ddp.all_reduce_(colsum)
                B_tot = B * ddp.world
                if ed_on:
                    feat_all, idx_all, B_all = ddp.all_gather(self._ed_feat), ddp.all_gather(idx), B_tot
            hip.call("es_router_loss", hip.ptr(gates), hip.ptr(idx) if ed_on else None,
                     hip.ptr(self._ed_feat) if ed_on else None, B, E, float(tau),
                     float(rc.alb_strength * dec_w), float(rc.util_strength), float(rc.ed_strength),
                     hip.ptr(colsum), B_tot, hip.ptr(feat_all), hip.ptr(idx_all), B_all,
                     hip.ptr(rl), hip.ptr(dlogits), hip.stream_ptr())
            if ddp is not None and ed_on:
                ddp.all_reduce_(rl[2:3])       # the ED sum over every rank's rows
            trained = epoch < rc.stop_router_training_epoch
            if trained:
                self.router.bwd(rctx, dlogits)
                # summed, not averaged: the router terms are functions of global sums
                self._allreduce(self.router, average=False)
                router_optimizer.step()
            flags = (1 | (2 if trained else 0) | (4 if rc.alb_strength != 0 else 0)
                     | (8 if rc.util_strength != 0 else 0) | (16 if ed_on else 0))

        self.step_count += 1
        self._eager_steps += 1
        hip.call("es_counter_add", hip.ptr(self._dstep), 1, hip.stream_ptr())
        # the metric dict (moe.py:480-502): one kernel over the expert rows and router terms
        countsf = None
        if self.ddp is not None:
            countsf = plan["gcnt"] if plan is not None else self.ddp.global_counts_tensor(dev)
        mvec = torch.empty(11 + 8 * E, dtype=torch.float32, device=dev)
        hip.call("es_step_metrics", hip.ptr(mbuf), E, hip.ptr(rl), hip.ptr(counts) if countsf is None else None,
                 hip.ptr(countsf), float(rc.gan_strength), float(rc.diff_strength), float(dec_w), flags,
                 hip.ptr(mvec), hip.stream_ptr())
        names = ["gen_loss", "disc_loss", "div_loss", "intensity_loss", "aux_reg_loss", "router_loss",
                 "expert_distribution_loss", "differentiation_loss", "expert_entropy_loss",
                 "adaptive_load_balancing_loss", "gan_loss"]
        for i in range(E):
            names += [f"gen_loss_{i}", f"disc_loss_{i}", f"div_loss_experts_{i}", f"intensity_loss_experts_{i}",
                      f"aux_reg_loss_experts_{i}", f"std_intensities_experts_{i}", f"mean_intensities_experts_{i}",
                      f"n_choosen_experts_mean_epoch_{i}"]
        return {k: mvec[j] for j, k in enumerate(names)}

    # ---------------------------------------------------------------------------- one expert
    # auto: concurrent experts while E x B capacity images of activations stay below this many
    # (each concurrent expert holds its own capacity-B buffers); serial experts share one set
    SERIAL_EXPERT_IMAGES = 16384

    def _experts_concurrent(self, E, B):
        """Run the experts' programs concurrently (own streams / graphs / memory) or one after another
        (one stream, buffers reused from expert to expert: activation memory of one capacity-B program
        instead of E).  train.expert_streams: auto | concurrent | serial."""
        if not self.expert_graphs_concurrent:
            return False
        mode = str(cfg_get(self.cfg, "train.expert_streams", "auto"))
        if mode not in ("auto", "concurrent", "serial"):
            raise ValueError(f"train.expert_streams must be auto, concurrent or serial, got {mode!r}")
        if mode == "auto":
            return E * B <= self.SERIAL_EXPERT_IMAGES
        return mode == "concurrent"

    def _fork_streams(self, E):
        """One side stream per expert (kept across steps), each made to wait for the current stream.
        (Measured, E = 4 B = 512 fp32: 2 / 3 / 4 streams 31.4 / 32.8 / 28.9 ms per step; 8 hardware
        queues instead of 4: 35.3 ms.)"""
        if getattr(self, "_side", None) is None or len(self._side) < E:
            self._side = [torch.cuda.Stream() for _ in range(E)]
        cur = torch.cuda.current_stream()
        for st in self._side[:E]:
            st.wait_stream(cur)
        return self._side[:E]

    def _bits_stream(self, e, G):
        """Side stream of expert e for the ahead-of-time dropout draw (train.dropout_ahead), or None
        (switched off, a generator without keep_plan / draw_keep, or several experts: a whole-step
        capture with the experts forked AND the draw forked from each expert's stream ended in a
        segmentation fault in capture_end, tools/gpu_r06r.sh; the draw measured slower anyway)."""
        if (not bool(cfg_get(self.cfg, "train.dropout_ahead", False)) or not hasattr(G, "draw_keep")
                or self.n_experts > 1):
            return None
        if getattr(self, "_bits_side", None) is None:
            self._bits_side = {}
        st = self._bits_side.get(e)
        if st is None:
            st = self._bits_side[e] = torch.cuda.Stream()
        return st

    def _plan(self, counts, B, dev):
        """The multi-expert step plan on the device (es_expert_plan): per expert the live rows of this
        process, the active flag (global count > 1, moe.py:126), the first global sample index, the
        loss weight count/B (moe.py:99-100), the global and live counts.  Data parallel: the ranks'
        counts are all-gathered on the device first (ddp.py)."""
        E, ddp = self.n_experts, self.ddp
        buf = lambda name, dt: self._buf(name, (E,), dt, dev)
        plan = {k: buf("plan_" + k, torch.int32) for k in ("rows", "active", "n0")}
        plan.update({k: buf("plan_" + k, torch.float32) for k in ("w", "gcnt", "lcnt")})
        counts_all, world, rank, min_local = None, 1, 0, 2
        if ddp is not None:
            counts_all = ddp.all_gather(counts)
            world, rank = ddp.world, ddp.rank
            # a rank with too few local samples trains with zero rows (zero local gradients, the
            # same collectives); SyncBN runs any non-empty shard (global statistics)
            min_local = 1 if ddp.sync_bn else 2
            ddp.set_plan(plan, B)
        hip.call("es_expert_plan", hip.ptr(counts), hip.ptr(counts_all), world, rank, E, B, min_local,
                 *[hip.ptr(plan[k]) for k in ("rows", "active", "n0", "w", "gcnt", "lcnt")], hip.stream_ptr())
        return plan

    def _expert_step(self, e, rows, be, B, cond, real, pos, std, intensity, opt_g, opt_d, opt_a, mbuf, step, dev,
                     plan=None):
        """plan (multi-expert steps): dynamic rows -- be = B is the capacity, the live count
        plan["rows"][e] is read on the device."""
        G, D, A = self.generators[e], self.discriminators[e], self.aux_regs[e]
        H, W = real.shape[2], real.shape[3]
        ridx = None
        live = None if plan is None else plan["rows"][e:e + 1]
        if rows is None:
            sc, sr, sp, ss, si = cond, real, pos, std, intensity
        else:
            # expert e's rows: perm[offs[e] : offs[e] + be] of the device dispatch, read at run time
            # (dynamic rows: the first live[0] of them, the rest of the capacity zero-filled)
            perm, offs = rows
            ridx = (perm, offs[e:e + 1])
            gather = lambda t, cols: _gather_rows(t, ridx, be, cols, live)
            sc, sp, ss, si = gather(cond, cond.shape[1]), gather(pos, 2), gather(std, 1), gather(intensity, 1)
            sr = gather(real.reshape(B, -1), H * W).view(be, 1, H, W)
        # class_counts_adjusted[i] as float32 (moe.py:99-100,522,562)
        # (DDP: local weight B_e^r / B_r; the all-reduce averages, see expertsim/train/ddp.py)
        w_dev = self._weight_scalar(be, B, dev) if plan is None else plan["w"][e:e + 1]
        # the step term (step * 1024) is added on the device from self._dstep
        sb = lambda pid: philox.dropout_stream(0, e, pid, 0)
        seed = self.rng_seed
        ddp = self.ddp
        n0 = 0                                                  # first global sample index
        if ddp is not None:
            n0 = ddp.sample_offset(e) if plan is None else plan["n0"][e:e + 1]
        sync = ddp is not None and ddp.sync_bn
        # data parallel: the expert's collectives (SyncBN, SDI mean, gradient buckets) run on its own
        # communicator when the experts run concurrently (ddp.expert_groups), else on the main group
        scope = ddp.on_expert(e) if ddp is not None else contextlib.nullcontext()
        with scope:
            if sync:
                set_norm_sync(ddp)
            try:
                if plan is None:
                    self._expert_program(e, be, B, G, D, A, sc, sr, sp, ss, si, opt_g, opt_d, opt_a, mbuf, dev,
                                         w_dev, sb, seed, n0, sync, rows, ridx, None, None)
                else:
                    with hip.live_rows(be, live, plan["active"][e:e + 1]), batch_live_counts():
                        self._expert_program(e, be, B, G, D, A, sc, sr, sp, ss, si, opt_g, opt_d, opt_a, mbuf,
                                             dev, w_dev, sb, seed, n0, sync, rows, ridx, live, plan["gcnt"][e:e + 1])
            finally:
                set_norm_sync(None)

    def _expert_program(self, e, be, B, G, D, A, sc, sr, sp, ss, si, opt_g, opt_d, opt_a, mbuf, dev, w_dev, sb,
                        seed, n0, sync, rows, ridx, live, gcnt):
        """live / gcnt (dynamic rows): the device live count and global count of the expert."""
        ddp = self.ddp

        # ---- generator forward #1 (moe.py:144-145)
        n1 = self._noise(e, 0, (be, self.noise_dim), dev, row0=n0)
        fake1, gctx1 = G.fwd(n1, sc, seed=seed, stream_base=sb(philox.PASS_G1), n_offset=n0)
        # train.dropout_ahead (off by default, measured 0.3-0.5 ms per step slower): the second forward's
        # dropout masks are data-independent, drawn on a side stream during the discriminator step and
        # read by that forward's norm passes
        pre2, bits_side = {}, self._bits_stream(e, G)
        if bits_side is not None:
            pre2 = {"pre": G.keep_plan(be, dev, seed=seed, stream_base=sb(philox.PASS_G2), n_offset=n0)}
            bits_side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(bits_side):
                G.draw_keep(pre2["pre"], be)

        # ---- discriminator step (moe.py:506-527)
        ro, _, dctx_r = D.fwd(Act.of(sr), sc)
        fo, _, dctx_f = D.fwd(fake1, sc)
        dro = torch.empty(be, 1, dtype=torch.float32, device=dev)
        dfo = torch.empty(be, 1, dtype=torch.float32, device=dev)
        hip.call("es_hinge_d", ro.ptr, fo.ptr, be, hip.ptr(live), hip.ptr(w_dev), hip.ptr(mbuf[e, 8:9]),
                 hip.ptr(dro), hip.ptr(dfo), hip.stream_ptr())
        D.bwd(dctx_r, dout=Act.of(dro), weight_grads=True, input_grad=False)
        D.bwd(dctx_f, dout=Act.of(dfo), weight_grads=True, input_grad=False)
        n2 = self._noise(e, 1, (be, self.noise_dim), dev, row0=n0)
        if bits_side is not None:
            torch.cuda.current_stream().wait_stream(bits_side)
        if ddp is None:
            opt_d.step()
            # ---- generator step (moe.py:529-571)
            fake2, gctx2 = G.fwd(n2, sc, seed=seed, stream_base=sb(philox.PASS_G2), n_offset=n0, **pre2)
        else:
            # data parallel: D's gradient all-reduce overlaps the second generator forward (which
            # does not read D); D's Adam waits for it
            ddp.allreduce_async(D)
            fake2, gctx2 = G.fwd(n2, sc, seed=seed, stream_base=sb(philox.PASS_G2), n_offset=n0, **pre2)
            ddp.wait_all()
            opt_d.step()
        fo1, fl1, dctx1 = D.fwd(fake1, sc)
        _, fl2, dctx2 = D.fwd(fake2, sc)
        s = torch.empty(be, dtype=torch.float32, device=dev)
        hip.call("es_image_expsum", C.byref(fake1.view), fake1.dt, fake1.ptr, hip.ptr(s), hip.stream_ptr())
        if self._ed_feat is not None:
            if rows is None:
                hip.call("es_scatter_rows", hip.ptr(s), None, be, hip.ptr(self._ed_feat), hip.stream_ptr())
            else:
                hip.call("es_scatter_rows_at", hip.ptr(s), hip.ptr(ridx[0]), hip.ptr(ridx[1]), be, hip.ptr(live),
                         hip.ptr(self._ed_feat), hip.stream_ptr())
        coords, actx = A.fwd(fake1, seed=seed, stream_base=sb(philox.PASS_AUX), n_offset=n0)
        L = fl1.dims[1]
        p = hip.GenLoss()
        p.n, p.latent, p.noise = be, L, self.noise_dim
        p.di_strength, p.in_strength = float(G.di_strength), float(G.in_strength)
        p.aux_strength = float(self.cfg.model.aux_reg.strength)
        p.rows = live.data_ptr() if live is not None else None
        if sync:
            # SDI prefactor mean(std)^2 over the expert's global batch (moe.py:573-588)
            std_mean = torch.empty(1, dtype=torch.float32, device=dev)
            hip.call("es_router_colsum", hip.ptr(ss), be, 1, hip.ptr(std_mean), hip.stream_ptr())
            ddp.all_reduce_(std_mean)
            if gcnt is not None:     # dynamic rows: / the expert's global count (device)
                hip.call("es_div_by", hip.ptr(std_mean), 1, hip.ptr(gcnt), hip.stream_ptr())
            else:
                sm = Act(std_mean, (1, 1, 1, 1), (1, 1, 1, 1), sample=False)
                copy_act(sm, sm, 1.0 / ddp.global_count(e), 0.0)
            p.std_mean = std_mean.data_ptr()
        dfo1 = torch.empty(be, 1, dtype=torch.float32, device=dev)
        dl1 = torch.empty(be, L, dtype=torch.float32, device=dev)
        dl2 = torch.empty(be, L, dtype=torch.float32, device=dev)
        dcoord = torch.empty(be, 2, dtype=torch.float32, device=dev)
        coef = torch.empty(be, dtype=torch.float32, device=dev)
        hip.call("es_gen_losses", C.byref(p), fo1.ptr, fl1.ptr, fl2.ptr, hip.ptr(n1), hip.ptr(n2), hip.ptr(ss),
                 hip.ptr(s), hip.ptr(si), coords.ptr, hip.ptr(sp), hip.ptr(w_dev), hip.ptr(mbuf[e, 0:8]),
                 hip.ptr(dfo1), hip.ptr(dl1), hip.ptr(dl2), hip.ptr(dcoord), hip.ptr(coef), hip.stream_ptr())
        dimg1 = D.bwd(dctx1, dout=Act.of(dfo1), dlat=Act.of(dl1), weight_grads=False, input_grad=True)
        dimg2 = D.bwd(dctx2, dout=None, dlat=Act.of(dl2), weight_grads=False, input_grad=True)
        dimga = A.bwd(actx, Act.of(dcoord), input_grad=True)
        if ddp is not None:
            ddp.allreduce_async(A)           # overlaps the generator backward
        copy_act(dimga, dimg1, 1.0, 1.0)
        hip.call("es_image_expsum_bwd", C.byref(fake1.view), fake1.dt, fake1.ptr, hip.ptr(coef),
                 C.byref(dimg1.view), dimg1.ptr, 1.0, hip.stream_ptr())
        G.bwd(gctx1, dimg1)
        # data parallel: the second backward finalises G's gradients layer by layer; each >= 1 MB
        # bucket is all-reduced while the remaining layers' backward runs
        G.bwd(gctx2, dimg2, ready=ddp.bucketer(G) if ddp is not None else None)
        if ddp is not None:
            ddp.wait_all()
        opt_g.step()
        opt_a.step()

    # ---------------------------------------------------------------------------- evaluation
    # generator batch of the evaluation (the reference uses 64, train/utils.py:118; eval-mode
    # outputs are per-sample, so the batch only sets how many images one HIP program covers)
    eval_batch_size = 1024

    @torch.no_grad()
    def evaluate(self, epoch, y_test, x_test, true_positions, std, intensity, cfg, device):
        """Wasserstein metrics of one test batch — reference moe.py:644-692.

        Real 5-channel sums: expm1 + masked sums of x_test on the device (es_channel_sums, one pass).
        Routing: the router with its stochastic Gumbel at tau=1 (moe.py:650), argmax.
        Generated sums: each expert's generator in eval mode over its routed conditions, images kept
        in HBM and reduced by the same kernel; WS distances on the host (train/utils.py:117-176).
        Returns {'ws_mean', 'ws_std', 'ws_mean_i', 'ws_std_i', 'epoch'}."""
        from ..train.utils import calculate_joint_ws_across_experts, channel_sums
        shape = tuple(cfg.dataset.input_image_shape)
        x = x_test if isinstance(x_test, torch.Tensor) else torch.as_tensor(np.asarray(x_test))
        x = x.reshape(-1, *shape)
        ch_org_dev = channel_sums(x.to(device, dtype=torch.float32), log_domain=True)
        y = y_test.to(device) if isinstance(y_test, torch.Tensor) else torch.as_tensor(y_test, device=device)
        soft_gates, _ = self.router(y.float())
        pred = torch.argmax(soft_gates, 1).cpu().numpy()
        ch_org = ch_org_dev.cpu().numpy()
        idx = [np.where(pred == i)[0] for i in range(self.n_experts)]
        ch_org_experts = [ch_org[ix] if len(ix) else np.zeros((0, 5)) for ix in idx]
        idx_dev = [torch.as_tensor(ix, device=device, dtype=torch.long) for ix in idx]
        ws_mean, ws_std, ws_mean_exp, ws_std_exp = calculate_joint_ws_across_experts(
            min(epoch // 5 + 1, 5), [x[ix] for ix in idx], [y[ix] for ix in idx_dev], list(self.generators),
            ch_org, ch_org_experts, self.noise_dim, device, batch_size=self.eval_batch_size,
            n_experts=self.n_experts, shape_images=shape)
        log = {"ws_mean": ws_mean, **{f"ws_mean_{i}": ws_mean_exp[i] for i in range(self.n_experts)},
               "ws_std": ws_std, **{f"ws_std_{i}": ws_std_exp[i] for i in range(self.n_experts)}, "epoch": epoch}
        return log

    def get_expert_assignment_counts(self, expert_assignments: torch.Tensor) -> torch.Tensor:
        counts = torch.bincount(expert_assignments.long(), minlength=self.n_experts).float()
        return counts / expert_assignments.size(0)


def _gather_rows(t: torch.Tensor, ridx, rows: int, cols: int, live=None) -> torch.Tensor:
    """ridx = (dispatch permutation, device start position): rows perm[start : start + rows]; with
    live (device int32 [1]) only the first live[0] rows, the rest zeros."""
    perm, start = ridx
    out = torch.empty(rows, cols, dtype=torch.float32, device=t.device)
    src = t.reshape(t.shape[0], -1)
    hip.call("es_gather_rows_at", hip.ptr(src), src.stride(0), hip.ptr(perm), hip.ptr(start), rows, cols,
             hip.ptr(out), cols, hip.ptr(live), hip.stream_ptr())
    return out


class ExpertGraphs:
    """HIP graphs of whole expert steps (gather, G fwd, D step + Adam, G step + Adam), one per
    (expert, batch size): the expert's rows are dynamic (its live count is read on the device), so one
    capture serves every routing.  A multi-expert step then issues ~40 launches from the
    host (router, dispatch, router loss + Adam, metrics) plus one graph replay per active expert,
    instead of ~450 launches per expert, and the experts' graphs run CONCURRENTLY, one HIP stream
    per expert: experts share no parameters and write disjoint rows of the step's buffers, and a
    quarter-batch expert alone leaves most of the chip idle.  Each expert has its own memory pool
    (its graphs replay one after another, so they may share temporaries; different experts'
    graphs may not; serial experts, concurrent=False, share one stream and one pool).  Everything
    that changes between steps is read on the device: the step
    counters (dropout / noise streams, Adam bias corrections), the expert's rows (dispatch
    permutation + device start + live count), the batch (static input buffers).  The first
    occurrence of a key is captured and then replayed; BatchNorm batch counts are advanced on the
    device inside the graph (gated on the expert's active flag)."""

    def __init__(self, max_graphs: int = 512, concurrent: bool = True):
        self.pools, self.streams = {}, {}
        self.concurrent = concurrent     # False: every expert's graph on one side stream (serialised)
        self.graphs = {}
        self.max_graphs = max_graphs
        self.captures = 0
        self.replays = 0
        self._used = []
        self._ready = None

    def clear(self):
        self.graphs = {}

    def begin(self):
        """Mark the point on the current stream the experts' graphs start after."""
        self._ready = torch.cuda.Event()
        self._ready.record()
        self._used = []

    def run(self, key, fn):
        from ..layers import count_batches, nbt_added, nbt_snapshot
        e = key[0]
        if e not in self.streams:
            # serial: every expert's graph replays on one stream, one after another, so they share
            # one memory pool too (a graph's temporaries are dead once its replay has finished)
            first = None if self.concurrent or not self.streams else next(iter(self.streams))
            self.streams[e] = self.streams[first] if first is not None else torch.cuda.Stream()
            self.pools[e] = self.pools[first] if first is not None else torch.cuda.graph_pool_handle()
        st = self.streams[e]
        st.wait_event(self._ready)
        entry = self.graphs.get(key)
        if entry is None:
            if len(self.graphs) >= self.max_graphs:
                self.graphs = {}
            before = nbt_snapshot()
            # no capture while other experts' graphs are replaying: measured (tests/test_graph_gpu.py,
            # E = 3 with every expert captured in one step) a capture overlapping the concurrent
            # replays corrupted them (metrics of the other experts off at the 1e-2 level; bitwise
            # equal to the eager steps with this device synchronisation, which torch.cuda.graph's
            # own capture protocol also performs).  A capture happens once per (expert, B_e) key.
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            # capture on the expert's own stream (torch.cuda.graph's gc.collect + empty_cache per
            # capture cost ~10 ms; the experts' captures do not need them)
            with torch.cuda.stream(st):
                g.capture_begin(pool=self.pools[e])
                try:
                    fn()
                finally:
                    g.capture_end()
            # the capture recorded the host-side batch counts once; replays re-apply them
            entry = self.graphs[key] = (g, nbt_added(before))
            self.captures += 1
        else:
            self.replays += 1
            for t, k in entry[1]:
                count_batches(t, k)
        with torch.cuda.stream(st):
            entry[0].replay()
        self._used.append(st)

    def join(self):
        """The current stream waits for every expert graph of this step."""
        cur = torch.cuda.current_stream()
        for st in set(self._used):
            cur.wait_stream(st)
        self._used = []
