"""Per-step replay of the C4 stall fixture (ref_c4_hard.npz) on the GPU: ADMM counts, f_des difference to the
oracle, in-band exits / beyond 1e-8 / robust redos per step.  python tools/c4_hard_steps.py"""
import sys, numpy as np
sys.path.insert(0, '/root/repo')
from tests._golden import load
from distributed_aerial_transportation_amd import BatchedController, Forest, scenarios
d = load("ref_c4_hard.npz"); n = 6; J, K = d["f_des"].shape[:2]
eng = BatchedController("cadmm", n, J, scenarios.params_block(n))
eng.set_forests([Forest.seeded(int(s)) for s in d["forest_seed"]], np.arange(J, dtype=np.int32))
eng.set_state(d["x0"], np.zeros(J, dtype=np.int32))
prev = eng.work()
for k in range(K):
    r = eng.control(None, None)
    w = eng.work()
    rel = [np.max(np.abs(r.f_des[j] - d["f_des"][j, k])) / max(1, np.abs(d["f_des"][j, k]).max()) for j in range(J)]
    print(k, r.iters.tolist(), ["%.1e" % x for x in rel], "inband", w["inband_exits"] - prev["inband_exits"],
          "loose", w["inband_beyond_clarabel_tol"] - prev["inband_beyond_clarabel_tol"], "redo", w["robust_redos"] - prev["robust_redos"],
          "qps", w["qp_solves"] - prev["qp_solves"], flush=True)
    prev = w
    eng.rollout(10)
