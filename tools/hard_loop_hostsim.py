"""CPU proxy of tests/test_gpu_hard_stretch.py: the oracle's C-ADMM / DD outer loop with every agent QP
answered by the device code's host build (tests/hostsim) instead of the oracle IPM, compared with the
fixture (f_des per HL step, outer iteration counts).

    python tools/hard_loop_hostsim.py cadmm|dd [hostsim .so]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_aerial_transportation_amd import scenarios  # noqa: E402
from distributed_aerial_transportation_amd.system import RQPState, pack_state  # noqa: E402
from oracle import controllers as oc  # noqa: E402
from oracle import forest as of  # noqa: E402
from oracle import model as om  # noqa: E402
from oracle import scenarios as osc  # noqa: E402
from tests import hostsim as hs  # noqa: E402


def main():
    kind = sys.argv[1]
    if len(sys.argv) > 2:
        hs._lib = ctypes.CDLL(sys.argv[2])
    d = np.load(os.path.join(ROOT, "tests", "golden", f"ref_{kind}_hard.npz"))
    n = 3
    p = osc.params(n)
    prm = scenarios.params_block(n)
    np.random.seed(0)
    forest = of.Forest()
    ctl = (oc.CADMM if kind == "cadmm" else oc.DD)(p, osc.col_radius(n), forest)
    s = RQPState.unpack(d["x0"], n)
    st = om.State(s.R, s.w, s.xl, s.vl, s.Rl, s.wl, project=False)
    bad = [0]

    def cadmm_solve(self, i, s_, acc, env, rho):
        lam = self.lam[:, :, i].T.reshape(-1).copy()
        fbar = self.f_mean.T.reshape(-1).copy()
        f, status, it, ib = hs.qp_cadmm_ex(prm, n, pack_state(s_), np.concatenate(acc), env.lhs, env.rhs, i, lam, fbar,
                                           rho)
        if status == 0:
            self.prev_f[i] = f.reshape(n, 3).T.copy()
        else:
            bad[0] += 1
        return self.prev_f[i], None

    def dd_solve(self, i, s_, acc, env, cf, cF, cM):
        x, status, it = hs.qp_dd(prm, n, pack_state(s_), np.concatenate(acc), env.lhs, env.rhs, i,
                                 np.concatenate([cf, cF, cM]))
        if status == 0:
            self.prev[i] = (x[:3].copy(), x[3:6].copy(), x[6:9].copy())
        else:
            bad[0] += 1
        return self.prev[i], None

    oc.CADMM.solve_agent = cadmm_solve
    oc.DD.solve_agent = dd_solve
    worst = 0.0
    for k in range(d["f_des"].shape[0]):
        bad[0] = 0
        acc, _, _ = oc.desired_acceleration_forest(st, forest)
        f, stat = ctl.control(st, acc)
        ref = d["f_des"][k]
        rel = np.max(np.abs(f - ref)) / max(1.0, np.max(np.abs(ref)))
        worst = max(worst, rel)
        print(f"step {k:2d}: iters {stat.iter:3d} (ref {int(d['iters'][k]):3d})  f_des rel diff {rel:.2e}  "
              f"non-optimal QPs {bad[0]}", flush=True)
        for _ in range(10):
            fl, M = om.low_level_control(p, st, f)
            st.integrate(*om.forward_dynamics(p, st, fl, M), 1e-3)
    print(f"worst f_des rel diff {worst:.2e}")


if __name__ == "__main__":
    main()
