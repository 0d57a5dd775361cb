"""Golden fixture ref_loose_caps.npz: the agent QPs the 10 s C4 loop accepted in band beyond Clarabel's 1e-8 (round 6,
before the robust solver's cone recovery), captured on the GPU by tools/capture_loose.py (a -DDAT_CAPTURE_LOOSE
build: scenario state, forest, acc_des, agent, the ADMM pass's multipliers, mean and rho), answered here by the
oracle's dense conic IPM (oracle/ipm.py) on the conic problem cvxpy would build (oracle/model.py::build_qp,
control/rqp_cadmm.py:376-501) at its own tolerance 1e-11 (x) and at Clarabel's 1e-8 (x_1e8: the spread two valid
solves of the reference show on these ill-determined QPs).  TEST infrastructure.

    python tests/golden/make_loose_caps.py gpurun_out/loose_caps.npz
"""
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from distributed_aerial_transportation_amd import Forest  # noqa: E402
from distributed_aerial_transportation_amd.system import RQPState  # noqa: E402
from oracle import forest as of  # noqa: E402
from oracle import model as om  # noqa: E402
from oracle import scenarios as osc  # noqa: E402
from oracle.ipm import solve_qp  # noqa: E402


def oforest(forest):
    """the oracle's forest object of a package Forest (tests/test_gpu_c4.py::_oforest)"""
    from tests.test_gpu_c4 import _oforest

    return _oforest(forest)


def main(src):
    warnings.filterwarnings("ignore")
    d = np.load(src)
    n = 6
    p = osc.params(n)
    c = om.Consts.make(p, osc.col_radius(n), distributed=True)
    feq = om.equilibrium_forces(p)
    K = len(d["agent"])
    x, x8, st = np.zeros((K, 3, n)), np.zeros((K, 3, n)), np.zeros(K, dtype=np.int32)
    for k in range(K):
        i = int(d["agent"][k])
        s0 = RQPState.unpack(d["state"][k], n)
        s = om.State(s0.R, s0.w, s0.xl, s0.vl, s0.Rl, s0.wl, project=False)
        env = of.env_rows(oforest(Forest.seeded(int(d["forest"][k]))), c, s, osc.col_radius(n), p.r[:, i])
        args = om.build_qp("cadmm", p, c, s, (d["acc"][k][:3], d["acc"][k][3:]), env, i=i, f_eq=feq,
                           lam=d["lam"][k].reshape(n, 3).T, rho=float(d["rho"][k]),
                           f_mean=d["fbar"][k].reshape(n, 3).T)
        r, r8 = solve_qp(*args), solve_qp(*args, tol=1e-8)
        x[k], x8[k], st[k] = r.x[9:].reshape(3, n, order="F"), r8.x[9:].reshape(3, n, order="F"), r.status
    np.savez_compressed(os.path.join(HERE, "ref_loose_caps.npz"), state=d["state"], forest=d["forest"],
                        acc=d["acc"], agent=d["agent"], lam=d["lam"], fbar=d["fbar"], rho=d["rho"],
                        admm_pass=d["admm_pass"], gpu_merit=d["merit"], x=x, x_1e8=x8, status=st)
    print(f"{K} QPs; oracle statuses {st.tolist()}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "loose_caps.npz"))
