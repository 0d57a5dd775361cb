"""Per-QP parity of the reduced agent-QP IPM (host build, tests/hostsim) along the oracle's C-ADMM / DD
hard stretch (tests/golden/ref_*_hard.npz): every agent QP the oracle solves is also solved by the
device code from the same inputs; failures and mismatches are counted per HL step and the failing
QPs are saved for replay.

    python tools/hard_qp_probe.py cadmm|dd [K] [out.npz]
"""
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
from oracle.ipm import OPTIMAL  # noqa: E402
from tests import hostsim as hs  # noqa: E402


def main():
    kind = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "diag", f"hard_{kind}_qps.npz")
    d = np.load(os.path.join(ROOT, "tests", "golden", f"ref_{kind}_hard.npz"))
    n = 3
    p = osc.params(n)
    prm = scenarios.params_block(n)
    np.random.seed(0)
    forest = of.Forest()
    ctl = (oc.CADMM if kind == "cadmm" else oc.DD)(p, osc.col_radius(n), forest)
    s = RQPState.unpack(d["x0"], n)
    st = om.State(s.R, s.w, s.xl, s.vl, s.Rl, s.wl, project=False)
    rec = {"step": [], "agent": [], "st": [], "acc": [], "lhs": [], "rhs": [], "lam": [], "fbar": [], "rho": [],
           "c9": [], "ref": [], "got": [], "status": [], "why": [], "iters": [], "oiters": []}
    step = [0]
    stats = {}

    def record(i, acc, env, ref, got, status, why, iters, oiters, lam=None, fbar=None, rho=1.0, c9=None):
        rec["step"].append(step[0]); rec["agent"].append(i); rec["st"].append(pack_state(st_cur[0]))
        rec["acc"].append(np.concatenate(acc)); rec["lhs"].append(env.lhs); rec["rhs"].append(env.rhs)
        rec["lam"].append(np.zeros(3 * n) if lam is None else lam); rec["fbar"].append(np.zeros(3 * n) if fbar is None else fbar)
        rec["rho"].append(rho); rec["c9"].append(np.zeros(9) if c9 is None else c9)
        rec["ref"].append(np.pad(ref, (0, 3 * n - ref.size))); rec["got"].append(np.pad(got, (0, 3 * n - got.size)))
        rec["status"].append(status); rec["why"].append(why); rec["iters"].append(iters); rec["oiters"].append(oiters)

    st_cur = [st]
    base_cadmm = oc.CADMM.solve_agent
    base_dd = oc.DD.solve_agent

    def tally(ok, bad_status, err):
        t = stats.setdefault(step[0], [0, 0, 0, 0.0])
        t[0] += 1
        t[1] += bad_status
        t[2] += (not bad_status) and err > 1e-5
        t[3] = max(t[3], err if not bad_status else 0.0)

    def cadmm_solve(self, i, s_, acc, env, rho):
        lam = self.lam[:, :, i].T.reshape(-1).copy()
        fbar = self.f_mean.T.reshape(-1).copy()
        out = base_cadmm(self, i, s_, acc, env, rho)
        r = self.last_r
        f, status, it, ib = hs.qp_cadmm_ex(prm, n, pack_state(s_), np.concatenate(acc), env.lhs, env.rhs, i, lam, fbar,
                                           rho)
        m, ib2, why = hs.last_diag()
        if r.status == OPTIMAL:
            ref = r.x[9:].reshape(3, n, order="F").T.reshape(-1)
            err = np.max(np.abs(f - ref)) / max(1.0, np.max(np.abs(ref)))
            bad = status != 0
            tally(True, bad, err)
            if bad or err > 1e-5 or ib:
                record(i, acc, env, ref, f, status + 100 * bool(ib), why, it, r.iters, lam, fbar, rho)
        return out

    def dd_solve(self, i, s_, acc, env, cf, cF, cM):
        out = base_dd(self, i, s_, acc, env, cf, cF, cM)
        r = self.last_r
        c9 = np.concatenate([cf, cF, cM])
        x, status, it = hs.qp_dd(prm, n, pack_state(s_), np.concatenate(acc), env.lhs, env.rhs, i, c9)
        m, ib, why = hs.last_diag()
        if r.status == OPTIMAL:
            ref = r.x[9:18]
            err = np.max(np.abs(x - ref)) / max(1.0, np.max(np.abs(ref)))
            bad = status != 0
            tally(True, bad, err)
            if bad or err > 1e-5 or ib:
                record(i, acc, env, ref, x, status + 100 * bool(ib), why, it, r.iters, c9=c9)
        return out

    # keep the oracle's result object of the last solve
    import oracle.controllers as occ

    orig = occ.solve_qp

    def solve_keep(*a, **k):
        r = orig(*a, **k)
        ctl.last_r = r
        return r

    occ.solve_qp = solve_keep
    oc.CADMM.solve_agent = cadmm_solve
    oc.DD.solve_agent = dd_solve
    for k in range(K):
        step[0] = k
        st_cur[0] = st
        acc, _, _ = oc.desired_acceleration_forest(st, forest)
        f, stat = ctl.control(st, acc)
        t = stats.get(k, [0, 0, 0, 0.0])
        print(f"step {k:2d}: outer it {stat.iter:3d}  QPs {t[0]:4d}  failed {t[1]:4d}  >1e-5 {t[2]:4d}  "
              f"max err {t[3]:.2e}", flush=True)
        for _ in range(10):
            fl, M = om.low_level_control(p, st, f)
            st.integrate(*om.forward_dynamics(p, st, fl, M), 1e-3)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    np.savez_compressed(out, **{k: np.array(v) for k, v in rec.items()})
    print("saved", len(rec["step"]), "records to", out)


if __name__ == "__main__":
    main()
