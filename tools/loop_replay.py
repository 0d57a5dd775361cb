"""Closed-loop replay from a recorded GPU state (diagnostic for the long-horizon tests).

    python tools/loop_replay.py gpu <controller> <record.npz> <k0> <K>   (GPU box: fresh handle, cold warm state)
    python tools/loop_replay.py cpu <controller> <record.npz> <k0> <K>   (oracle loop from the same state, compare)
controller: consensus-admm | dual-decomposition
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mode, ct, src, k0, K = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
x0 = np.load(src)["states"][k0]
n = 3
out = os.path.join(ROOT, "gpurun_out", f"replay_{ct[:4]}_{k0}.npz")
if mode == "gpu":
    from distributed_aerial_transportation_amd import BatchedController, Forest, scenarios

    eng = BatchedController(ct, n, 1, scenarios.params_block(n))
    eng.set_forests([Forest.seeded(0)])
    eng.set_state(x0[None], np.zeros(1, dtype=np.int32))
    F, I, QS = [], [], []
    for k in range(K):
        r = eng.control(None, None)
        F.append(r.f_des[0].copy()), I.append(r.iters[0]), QS.append(r.qp_status[0].copy())
        eng.rollout(10)
    np.savez(out, f_des=np.array(F), iters=np.array(I), qp_status=np.array(QS))
    print("iters", [int(i) for i in I])
else:
    from distributed_aerial_transportation_amd.system import RQPState
    from oracle import controllers as oc
    from oracle import forest as of
    from oracle import model as om
    from oracle import scenarios as osc

    r = np.load(out) if os.path.exists(out) else None
    p = osc.params(n)
    np.random.seed(0)
    forest = of.Forest()
    ctl = (oc.DD if ct == "dual-decomposition" else oc.CADMM)(p, osc.col_radius(n), forest)
    s = RQPState.unpack(x0, n)
    st = om.State(s.R, s.w, s.xl, s.vl, s.Rl, s.wl, project=False)
    for k in range(K):
        acc, _, _ = oc.desired_acceleration_forest(st, forest)
        f, stat = ctl.control(st, acc)
        line = f"step {k0 + k}: oracle iters {stat.iter:3d}"
        if r is not None:
            df = np.max(np.abs(f - r["f_des"][k])) / max(1.0, np.max(np.abs(f)))
            line += f" gpu {r['iters'][k]:3d}  f diff {df:.2e}  gpu status {r['qp_status'][k]}"
        print(line, flush=True)
        for _ in range(10):
            fl, M = om.low_level_control(p, st, f)
            st.integrate(*om.forward_dynamics(p, st, fl, M), 1e-3)
