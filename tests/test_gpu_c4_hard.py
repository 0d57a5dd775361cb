"""C4 stall stretches (tests/golden/make_c4_hard.py): n = 6 C-ADMM in seeded forests, from states the GPU's
own C4 10 s loop reached one HL step before their first stall.  From the second step on every step is the
reference controller's 101-pass ADMM stall (control/rqp_cadmm.py:631-675): the consensus multipliers grow
through the dual update (:627-629) and the agent QPs carry active rows and cones with barrier weights of
1e10-1e19.  There the round-4 solver accepted in-band iterates outside Clarabel's 1e-8 (22 and 48 over these
two stretches on the host build) and left the oracle's f_des by 2e-4 at steps 16-17 of the second.

The GPU loop (cold warm state, the production k_env_class -> k_cadmm / k_cadmm_rob path) must follow the
oracle through both stretches: ADMM iteration counts exact, and f_des within 1e-5 relative at every step --
or within the loop's own sensitivity to solver accuracy: 5 x the oracle's spread between QP tolerances 1e-10
and 1e-11 (f_des_1e10; 1.1e-2 at step 18 of the second stretch), or the spread at Clarabel's own tolerance
1e-8 (f_des_1e8: the reference's solver settings; the fast solver accepts in-band iterates within 1e-8 as
Clarabel would, and the reference run at 1e-8 moves by 1.9e-4 at step 16 of the second stretch).  No in-band
accept beyond Clarabel's 1e-8 (round 4 had 22 and 48 over the two stretches on the host build, round 5 up
to one per stretch; since round 6 the stalled passes run in the tail kernel)."""

import numpy as np
import pytest

from tests._golden import load

pytestmark = pytest.mark.gpu


def test_gpu_c4_stall_stretches_match_oracle():
    from distributed_aerial_transportation_amd import BatchedController, Forest, scenarios

    d = load("ref_c4_hard.npz")
    n = 6
    J, K = d["f_des"].shape[:2]
    eng = BatchedController("cadmm", n, J, scenarios.params_block(n))
    eng.set_forests([Forest.seeded(int(s)) for s in d["forest_seed"]], np.arange(J, dtype=np.int32))
    eng.set_state(d["x0"], np.zeros(J, dtype=np.int32))
    its = d["iters"].astype(int)
    assert np.all(its[:, 1:] == 101)
    worst = np.zeros(J)
    loose0 = eng.work()["inband_beyond_clarabel_tol"]
    for k in range(K):
        r = eng.control(None, None)
        np.testing.assert_array_equal(r.iters, its[:, k], err_msg=f"step {k}")
        for j in range(J):
            ref = d["f_des"][j, k]
            scale = max(1.0, np.max(np.abs(ref)))
            rel = np.max(np.abs(r.f_des[j] - ref)) / scale
            sens = np.max(np.abs(d["f_des_1e10"][j, k] - ref)) / scale
            sens8 = np.max(np.abs(d["f_des_1e8"][j, k] - ref)) / scale
            assert rel < max(1e-5, 5.0 * sens, sens8), (j, k, rel, sens, sens8)
            worst[j] = max(worst[j], rel if sens < 1e-5 else 0.0)
        eng.rollout(10)
    w = eng.work()
    loose = w["inband_beyond_clarabel_tol"] - loose0
    print(f"C4 stall stretches: {J} x {K} steps, iteration counts exact; largest f_des difference where the "
          f"reference is reproducible {worst.max():.2e}; in-band accepts beyond 1e-8: {loose}; robust redos "
          f"{w.get('robust_redos', 0)}")
    assert loose == 0


def test_gpu_c4_stall_sub_batches_bitwise():
    """The wedged scenarios' steps do not depend on the schedule: with one sub-batch k_env_class routes them to
    the tail launch beside k_cadmm (KArgs::route), with two k_cadmm hands them over before their first pass
    (dat.hip cadmm_drain, `wedged`); both runs of the closed loop (the stretches' 2 scenarios twice) end bitwise
    equal after 3 HL steps, the last two of them 101-pass stalls."""
    from distributed_aerial_transportation_amd import BatchedController, Forest, scenarios

    d = load("ref_c4_hard.npz")
    n = 6
    J = d["x0"].shape[0]
    x0 = np.concatenate([d["x0"], d["x0"]])
    sf = np.concatenate([np.arange(J), np.arange(J)]).astype(np.int32)
    out = []
    for nsub in (1, 2):
        eng = BatchedController("cadmm", n, 2 * J, scenarios.params_block(n))
        try:
            eng.set_forests([Forest.seeded(int(s)) for s in d["forest_seed"]], sf)
            eng.set_state(x0, np.zeros(2 * J, dtype=np.int32))
            eng.set_sub_batches(nsub)
            eng.closed_loop(3)
            eng.synchronize()
            st, _ = eng.get_state()
            out.append((st, eng.work()))
        finally:
            eng.close()
    (s1, w1), (s2, w2) = out
    assert w1["tail_routed"] > 0 and w2["tail_routed"] == 0
    assert np.array_equal(s1, s2)
    assert np.array_equal(s1[:J], s1[J:])
