"""Closed-loop parity over the reference horizon, through the reference's log format.

example/rqp_example.py:main (T = 100 s, dt = 1e-3, HL every 10 steps, forest seed 0, LL "pd") run on
the GPU by ``example.simulate_batch`` against the reference's own loop (ref_long_<tag>.npz, written
by tests/golden/make_golden.py from the reference code): centralized and C-ADMM over the full 100 s,
DD over 10 s (its reference loop runs up to 101 x 3 agent solves per HL step).  Every logged quantity
is compared (f_des_seq, iter_seq, min_env_dist_seq per HL step; x_err_seq / v_err_seq per log step;
state_seq and w_seq every 10th log step).  north_star: closed-loop states within 1e-4 over the
horizon; the test reports the first HL step at which f_des leaves 1e-5 or a state leaves 1e-4 (the
divergence onset) and requires that there is none.
"""

import os

import numpy as np
import pytest

from tests._golden import GOLDEN, load, unpack_flat

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


@pytest.mark.timeout(900)
@pytest.mark.parametrize("tag,ct", [("cent", "centralized"), ("cons", "consensus-admm"), ("dual", "dual-decomposition")])
def test_gpu_long_closed_loop_logs(tag, ct, capsys):
    from distributed_aerial_transportation_amd import Forest, example, scenarios, system

    name = f"ref_long_{tag}.npz"
    if not os.path.exists(os.path.join(GOLDEN, name)):
        pytest.skip(f"{name} not generated yet (python -O tests/golden/make_golden.py long {ct})")
    d = load(name)
    T, every = float(d["T"]), int(d["state_every"])
    _, _, s0 = scenarios.rqp_setup(3)
    logs = example.simulate_batch(ct, system.pack_state(s0)[None], [Forest.seeded(0)], n=3, T=T)[0]
    K = d["f_des"].shape[0]
    assert len(logs["f_des_seq"]) == K and len(logs["x_err_seq"]) == d["x_err"].shape[0]
    assert len(logs["state_seq"]) == d["x_err"].shape[0] and len(logs["w_seq"]) == d["x_err"].shape[0]
    assert logs["num_trees"] == 128 and logs["controller_type"] == ct and logs["log_freq"] == 10
    f = np.array(logs["f_des_seq"])
    df = np.array([_rel(f[k], d["f_des"][k]) for k in range(K)])
    xs = np.array([system.pack_state(s) for s in logs["state_seq"][::every]])
    ref = np.array([system.pack_state(unpack_flat(x, 3)) for x in d["states"]])
    ds = np.max(np.abs(xs - ref), axis=1)
    onset_f = int(np.argmax(df > 1e-5)) if np.any(df > 1e-5) else None
    onset_s = int(np.argmax(ds > 1e-4)) * every if np.any(ds > 1e-4) else None
    with capsys.disabled():
        print(f"\n[{ct}] T = {T:.0f} s, {K} HL steps: max f_des rel diff {df.max():.2e}, max state diff {ds.max():.2e}; "
              f"divergence onset (HL step): f_des {onset_f}, state {onset_s}")
    assert onset_f is None and onset_s is None
    if ct != "centralized":
        np.testing.assert_array_equal(np.array(logs["iter_seq"]), d["iters"])
    else:
        assert logs["iter_seq"] == []
    np.testing.assert_allclose(logs["min_env_dist_seq"], d["min_dist"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(logs["x_err_seq"], d["x_err"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(logs["v_err_seq"], d["v_err"], rtol=0, atol=1e-4)
    w = np.array([np.concatenate([fw.reshape(-1), Mw.reshape(-1)]) for fw, Mw in logs["w_seq"][::every]])
    np.testing.assert_allclose(w, d["w"], rtol=0, atol=1e-4)
    # the statistics printout of example/rqp_example.py:62-80
    example.print_stats(logs["iter_seq"], logs["solve_time_seq"])
    out = capsys.readouterr().out
    assert "Solver solve time (ms): min:" in out
    if ct != "centralized":
        assert out.startswith("Solver iterations: min:")
