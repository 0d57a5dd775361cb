"""The C4 closed-loop fixture's own reproducibility horizon (CPU, dev container): re-run
make_golden.gen_c4_loop (the reference's loop behind tests/golden/refstubs.py) with the oracle IPM
tolerance changed 1e-11 -> `tol` and write ref_c4_loop.npz to /tmp, for tests/golden/c4_horizon.json.

    python -O tools/c4_sensitivity.py 1e-10
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)
tol = float(sys.argv[1])
import oracle.ipm as oipm  # noqa: E402

_orig = oipm.solve_qp
oipm.solve_qp = lambda *a, **k: _orig(*a, **{**k, "tol": tol})
import make_golden as mg  # noqa: E402

mg.gen_c4_loop(out_dir="/tmp")
