"""Fixtures ref_dd_hard.npz / ref_cadmm_hard.npz: hard closed-loop stretches from one state, answered
by the oracle (oracle/controllers.py DD / CADMM, pinned to the reference's loops by
tests/test_oracle_golden.py).  Past the reference loop's own reproducibility horizon
(tools/long_sensitivity.py) the GPU's and the reference's runs of example/rqp_example.py (forest seed
0) part, and the GPU trajectory reaches states from which the controller itself fails:
  dd     x0 = HL step 4290 of the GPU DD loop: the dual ascent climbs 12 -> 59 iterations and stalls
         at max_iter for seven steps (control/rqp_dd.py:741-752), 40 steps recorded;
  cadmm  x0 = HL step 5595 of the GPU C-ADMM loop: next to a tree the ADMM loop stalls at max_iter
         from step 5606 on (control/rqp_cadmm.py:631-675), 16 steps recorded.
The oracle does exactly what the GPU does from these states (tests/test_gpu_hard_stretch.py).
The run is recorded twice: at the oracle's QP tolerance (1e-11, f_des) and at 1e-10 (f_des_1e10), whose
difference is the loop's own sensitivity to solver accuracy inside a stall (DD: up to 7.6e-5 relative).

    python tests/golden/make_hard_stretch.py dd|cadmm [<npz with states (GPU long-loop record)> <k0>]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from distributed_aerial_transportation_amd.system import RQPState  # noqa: E402
from oracle import controllers as oc  # noqa: E402
from oracle import forest as of  # noqa: E402
from oracle import model as om  # noqa: E402
from oracle import scenarios as osc  # noqa: E402

CASES = {"dd": ("ref_dd_hard.npz", 40, oc.DD), "cadmm": ("ref_cadmm_hard.npz", 16, oc.CADMM)}


def run(ctor, x0, K, tol):
    import oracle.controllers as occ

    orig = occ.solve_qp
    occ.solve_qp = lambda *a, **k: orig(*a, tol=tol, **k)
    try:
        n = 3
        p = osc.params(n)
        np.random.seed(0)
        forest = of.Forest()
        ctl = ctor(p, osc.col_radius(n), forest)
        s = RQPState.unpack(x0, n)
        st = om.State(s.R, s.w, s.xl, s.vl, s.Rl, s.wl, project=False)
        F, I = [], []
        for k in range(K):
            acc, _, _ = oc.desired_acceleration_forest(st, forest)
            f, stat = ctl.control(st, acc)
            F.append(f.copy()), I.append(stat.iter)
            print(tol, k, stat.iter, flush=True)
            for _ in range(10):
                fl, M = om.low_level_control(p, st, f)
                st.integrate(*om.forward_dynamics(p, st, fl, M), 1e-3)
    finally:
        occ.solve_qp = orig
    return np.array(F), np.array(I, dtype=np.int16)


def main():
    OUT, K, ctor = CASES[sys.argv[1]]
    OUT = os.path.join(HERE, OUT)
    if len(sys.argv) > 3:
        x0 = np.load(sys.argv[2])["states"][int(sys.argv[3])]
    else:
        x0 = np.load(OUT)["x0"]
    F, I = run(ctor, x0, K, 1e-11)
    F10, _ = run(ctor, x0, K, 1e-10)
    np.savez_compressed(OUT, x0=x0, f_des=F, iters=I, f_des_1e10=F10)


if __name__ == "__main__":
    main()
