"""Stage-by-stage probe of the data-parallel multi-expert step at RCCL world size 1 (diagnostics:
prints each stage, dumps every thread's stack if a stage stalls).
usage: python tools/ddp_e4_probe.py [E] [B] [own_groups 0/1] [fork 0/1]"""
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "generative-dnn-for-physics-simulations-cern_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

faulthandler.dump_traceback_later(40, repeat=True, exit=False)
E = int(sys.argv[1]) if len(sys.argv) > 1 else 4
B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
own = int(sys.argv[3]) if len(sys.argv) > 3 else 1
fork = int(sys.argv[4]) if len(sys.argv) > 4 else 1
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
import bench  # noqa: E402
from expertsim.train.ddp import DataParallel  # noqa: E402
from expertsim.utils.synthetic import make_batch  # noqa: E402
from expertsim.graph import StepGraph  # noqa: E402


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


b = make_batch(B, "neutron", seed=5)
t = {k: torch.from_numpy(v).to(dev) for k, v in b.items()}
real = t["real_images"].unsqueeze(1).contiguous()
moe, (og, od, oa, orr), cfg = bench.build("neutron", E, "fp32", 1234, dev)
moe.ddp = DataParallel(sync_bn=True)
if not fork:
    cfg.train.expert_streams = "serial"
if not own:
    moe.ddp.ensure_expert_groups = lambda E: None
args = (0, t["cond"], real, t["true_positions"], t["std"], t["intensity"], oa, og, od, orr, None, dev)
for i in range(3):
    log("eager step", i, "issue")
    m = moe.train_step(*args)
    log("eager step", i, "issued; synchronising")
    torch.cuda.synchronize()
    log("eager step", i, "done", float(m["gen_loss"]))
log("capture")
sg = StepGraph(moe, args, warmup=0)
log("captured; replay")
for i in range(2):
    sg.replay()
    torch.cuda.synchronize()
    log("replay", i, "done", float(sg.metrics["gen_loss"]))
dist.destroy_process_group()
log("ok")
