"""The agent QPs the 10 s C4 loop accepted in band beyond Clarabel's 1e-8 before the robust solver's cone recovery
(20 captured on the GPU by tools/capture_loose.py, answered by the oracle: tests/golden/make_loose_caps.py), solved
through the single-QP C-ABI surface (dat_solve_agent_qp_batch, the C-ADMM agent QP as the closed loop defines it):
every one OPTIMAL with no in-band accept beyond 1e-8, at the oracle's answer up to the oracle's own spread between
Clarabel's 1e-8 and its 1e-11 (these QPs carry active rows with barrier weights of 1e10 and more; the oracle's
answer moves by up to 2.5e-3 between the two tolerances)."""

import numpy as np
import pytest

from tests._golden import load
from tests.test_hostsim import _loose_bound

pytestmark = pytest.mark.gpu


def test_gpu_loose_caps_within_clarabel_tol():
    from distributed_aerial_transportation_amd import BatchedController, Forest, scenarios

    d = load("ref_loose_caps.npz")
    n, K = 6, len(d["agent"])
    fids = sorted(set(int(f) for f in d["forest"]))
    eng = BatchedController("cadmm", n, K, scenarios.params_block(n))
    eng.set_forests([Forest.seeded(f) for f in fids], np.array([fids.index(int(f)) for f in d["forest"]], np.int32))
    eng.set_state(d["state"], np.zeros(K, dtype=np.int32))
    w0 = eng.work()
    r = eng.solve_agent_qps(np.arange(K), d["agent"], d["acc"], lam=d["lam"].reshape(K, n, 3).transpose(0, 2, 1),
                            rho=d["rho"], f_mean=d["fbar"].reshape(K, n, 3).transpose(0, 2, 1))
    w = eng.work()
    assert np.all(r["status"] == 0), r["status"]
    assert w["inband_beyond_clarabel_tol"] - w0["inband_beyond_clarabel_tol"] == 0
    worst = 0.0
    for k in range(K):
        rel, bound = _loose_bound(d, k, r["x"][k])
        assert rel < bound, (k, rel, bound)
        worst = max(worst, rel)
    print(f"{K} loose-accept QPs: all OPTIMAL within Clarabel's 1e-8; largest difference to the oracle {worst:.1e}")
