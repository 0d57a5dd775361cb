"""DD closed-loop replay from a recorded GPU state (diagnostic for test_gpu_long's DD loop).

    python tools/dd_replay.py gpu  <long_dual.npz> <k0> <K>   (GPU box: fresh handle, cold DD warm state)
    python tools/dd_replay.py cpu  <long_dual.npz> <k0> <K>   (oracle loop from the same state, compare)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mode, src, k0, K = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
g = np.load(src)
x0 = g["states"][k0]
n = 3
out = os.path.join(ROOT, "gpurun_out", f"dd_replay_{k0}.npz")
if mode == "gpu":
    from distributed_aerial_transportation_amd import BatchedController, Forest, scenarios

    eng = BatchedController("dual-decomposition", n, 1, scenarios.params_block(n))
    eng.set_forests([Forest.seeded(0)])
    eng.set_state(x0[None], np.zeros(1, dtype=np.int32))
    F, I, X, QS = [], [], [], []
    for k in range(K):
        X.append(eng.get_state()[0][0].copy())
        r = eng.control(None, None)
        F.append(r.f_des[0].copy()), I.append(r.iters[0]), QS.append(r.qp_status[0].copy())
        eng.rollout(10)
    np.savez(out, f_des=np.array(F), iters=np.array(I), states=np.array(X), qp_status=np.array(QS))
    print("iters", I)
else:
    from distributed_aerial_transportation_amd.system import RQPState
    from oracle import controllers as oc
    from oracle import forest as of
    from oracle import model as om
    from oracle import scenarios as osc

    r = np.load(out)
    p = osc.params(n)
    np.random.seed(0)
    forest = of.Forest()
    ctl = oc.DD(p, osc.col_radius(n), forest)
    s = RQPState.unpack(x0, n)
    st = om.State(s.R, s.w, s.xl, s.vl, s.Rl, s.wl, project=False)
    for k in range(K):
        acc, _, _ = oc.desired_acceleration_forest(st, forest)
        f, stat = ctl.control(st, acc)
        df = np.max(np.abs(f - r["f_des"][k])) / max(1.0, np.max(np.abs(f)))
        print(f"step {k0 + k}: oracle iters {stat.iter:3d} gpu {r['iters'][k]:3d}  f diff {df:.2e}  gpu status {r['qp_status'][k]}",
              flush=True)
        for _ in range(10):
            fl, M = om.low_level_control(p, st, f)
            st.integrate(*om.forward_dynamics(p, st, fl, M), 1e-3)
