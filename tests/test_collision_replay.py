"""The collisions of the sustained 10 s C4 loop (bench.py sustained_loop: 65,536 scenarios, 1,000 HL steps) are
the reference controller's own.  tests/golden/c4_collision.npz (tools/collision_replay.py, on the GPU): the loop's
only colliding scenario (27522, forest 2: 185 collided scenario-steps, every step from 815 on) from its state three
HL steps before its first collision, replayed with the warm state reset by the GPU's production path (f_des, ADMM
iterations, min env distance, collision flag per step).  Replayed in the oracle (oracle/controllers.CADMM, the
reference's C-ADMM controller restated, control/rqp_cadmm.py) from the same state, it collides at the same steps
with the same ADMM iteration counts (1-17 passes, no stall) and f_des within 1e-6: the collision flag
(example/env_forest.py:158-159) is raised on a trajectory the reference's controller produces, not by the GPU
path's numerics."""
import numpy as np
import pytest

from tests._golden import load

N = 6


def test_c4_collision_replayed_by_oracle():
    from distributed_aerial_transportation_amd.system import RQPState
    from oracle import controllers as oc
    from oracle import forest as of
    from oracle import model as om
    from oracle import scenarios as osc

    d = load("c4_collision.npz")
    assert int(d["scenario_steps"]) == 185 and int(d["n_collided"]) == 1
    p = osc.params(N)
    for q in range(len(d["ids"])):
        np.random.seed(int(d["forest"][q]))
        forest = of.Forest()
        x = RQPState.unpack(d["st0"][q], N)
        st = om.State(x.R, x.w, x.xl, x.vl, x.Rl, x.wl, project=False)
        ctl = oc.CADMM(p, osc.col_radius(N), forest)
        hits = []
        for k in range(d["f_des"].shape[0]):
            acc, _, _ = oc.desired_acceleration_forest(st, forest)
            f, stat = ctl.control(st, acc)
            ref = d["f_des"][k, q]
            assert stat.iter == d["iters"][k, q], (q, k)
            assert np.max(np.abs(f - ref)) / max(1.0, np.max(np.abs(ref))) < 1e-6, (q, k)
            assert stat.min_env_dist == pytest.approx(d["min_env_dist"][k, q], abs=1e-8), (q, k)
            assert bool(stat.collision) == bool(d["collision"][k, q]), (q, k)
            hits.append(bool(stat.collision))
            for _ in range(10):
                fl, M = om.low_level_control(p, st, f)
                st.integrate(*om.forward_dynamics(p, st, fl, M), 1e-3)
        # the collision three steps after the replay's start, as in the loop (its first at step s0 + 3)
        assert hits.index(True) == int(d["first"][q] - d["s0"][q])


@pytest.mark.gpu
def test_gpu_c4_collision_replay():
    """The production path replays the fixture bitwise-stably: the same ADMM iterations and collision flags, f_des
    within 1e-9 (the fixture was written by an earlier build of the same path)."""
    from distributed_aerial_transportation_amd import BatchedController, Forest, scenarios

    d = load("c4_collision.npz")
    ids = d["ids"]
    forests = [Forest.seeded(s) for s in range(64)]
    eng = BatchedController("cadmm", N, len(ids), scenarios.params_block(N))
    eng.set_qp_tolerance(1e-10)
    eng.set_forests(forests, d["forest"].astype(np.int32))
    eng.set_state(d["st0"], d["c0"])
    try:
        for k in range(d["f_des"].shape[0]):
            r = eng.control()
            ref = d["f_des"][k]
            assert np.array_equal(r.iters, d["iters"][k]), k
            assert np.array_equal(r.collision, d["collision"][k]), k
            assert np.max(np.abs(r.f_des - ref)) / max(1.0, np.max(np.abs(ref))) < 1e-9, k
            eng.rollout(10)
        # the device counters of the same steps (bench stats.sustained): collided scenario-steps and the signed
        # smallest env distance (negative: inside the tree)
        w = eng.work()
        assert w["collisions"] == int(d["collision"].sum())
        assert w["min_env_dist"] == pytest.approx(float(d["min_env_dist"].min()), abs=1e-9)
        assert w["min_env_dist"] < 0.0
    finally:
        eng.close()
