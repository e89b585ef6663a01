"""Debug: per-metric / per-parameter deviation of the 2-rank SyncBN step from the single-device step."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, "generative-dnn-for-physics-simulations-cern_amd")
sys.path.insert(0, ".")
import test_ddp_gpu as T

if __name__ == "__main__":
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    single, lr = T._run(E, T.B_GLOBAL)
    dp = T._spawn(E, True)[0]
    for s, ((ms, ps), (md, pd)) in enumerate(zip(single, dp)):
        bad = {k: (v, md[k]) for k, v in ms.items() if abs(md[k] - v) / max(abs(v), 1e-3) > 1e-4}
        print("step", s, "metrics off:", bad)
        worst = sorted(((float(np.max(np.abs(pd[n] - a))) / lr[n.split(".")[0]], n) for n, a in ps.items()))[-5:]
        print("step", s, "worst params / lr:", worst)
