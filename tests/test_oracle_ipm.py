"""The oracle's conic IPM (oracle/ipm.py) certified independently of itself.

Clarabel (the solver the reference calls, control/rqp_cadmm.py:492) is absent here, so the
oracle's answers are pinned by (i) their KKT certificate computed from scratch in this test and
(ii) an independent solver: scipy's SLSQP on the same problems (the SOCs as smooth constraints),
on the conic data the reference's own cvxpy model produced (tests/golden/ref_qp.npz).
"""

import numpy as np
import pytest
from scipy.optimize import minimize

from oracle.ipm import OPTIMAL, ConeDims, cone_violation, solve_qp
from tests._golden import load


def _problem(d, pre):
    G, h, l = d[pre + "G"], d[pre + "h"], int(d[pre + "l"])
    keep = np.ones(G.shape[0], bool)
    keep[:l] = np.any(G[:l] != 0, axis=1) | (h[:l] != 0)
    dims = ConeDims(l=int(keep[:l].sum()), q=[int(x) for x in d[pre + "q_dims"]])
    return d[pre + "P"], d[pre + "q"], G[keep], h[keep], dims, d[pre + "A"], d[pre + "b"]


def _kkt(P, q, G, h, dims, A, b, r):
    """Residuals of the KKT system, recomputed from the returned (x, y, z, s)."""
    rx = P @ r.x + q + A.T @ r.y + G.T @ r.z
    rp = G @ r.x + r.s - h
    ra = A @ r.x - b
    return (np.max(np.abs(rx)), max(np.max(np.abs(rp)), np.max(np.abs(ra))), float(r.s @ r.z),
            cone_violation(r.s, dims), cone_violation(r.z, dims))


CASES = [(k, c) for k in ("cadmm", "dd", "cen") for c in range(6)]


@pytest.mark.parametrize("kind,case", CASES)
def test_ipm_certificate(kind, case):
    d = load("ref_qp.npz")
    P, q, G, h, dims, A, b = _problem(d, f"{kind}{case}_")
    r = solve_qp(P, q, G, h, dims, A, b)
    assert r.status == OPTIMAL
    dres, pres, gap, sv, zv = _kkt(P, q, G, h, dims, A, b, r)
    scale = 1.0 + max(np.max(np.abs(q)), np.max(np.abs(h)))
    assert dres < 1e-9 * scale and pres < 1e-9 * scale and abs(gap) < 1e-9 * scale
    assert sv <= 1e-12 and zv <= 1e-12


@pytest.mark.parametrize("kind,case", [(k, c) for k, c in CASES if c < 3])
def test_ipm_matches_independent_solver(kind, case):
    d = load("ref_qp.npz")
    P, q, G, h, dims, A, b = _problem(d, f"{kind}{case}_")
    r = solve_qp(P, q, G, h, dims, A, b)

    def f(x):
        return 0.5 * x @ P @ x + q @ x, P @ x + q

    cons = [{"type": "eq", "fun": lambda x: A @ x - b, "jac": lambda x: A}]
    if dims.l:
        cons.append({"type": "ineq", "fun": lambda x: (h - G @ x)[: dims.l], "jac": lambda x: -G[: dims.l]})
    for off, k in dims.blocks():
        def soc(x, off=off, k=k):
            s = h[off : off + k] - G[off : off + k] @ x
            return s[0] ** 2 - s[1:] @ s[1:]  # with s[0] >= 0 below: s in the cone

        cons.append({"type": "ineq", "fun": soc})
        cons.append({"type": "ineq", "fun": lambda x, off=off: h[off] - G[off] @ x})
    x0 = np.linalg.lstsq(A, b, rcond=None)[0]
    res = minimize(f, x0, jac=True, constraints=cons, method="SLSQP", options={"ftol": 1e-14, "maxiter": 500})
    # status 8 = SLSQP stopped at its own line-search precision limit; judged by the checks below
    assert res.status in (0, 8), res.message
    obj_ipm = 0.5 * r.x @ P @ r.x + q @ r.x
    assert res.fun == pytest.approx(obj_ipm, rel=1e-7, abs=1e-8)
    # strictly convex: the minimiser is unique
    np.testing.assert_allclose(res.x, r.x, atol=2e-5)
