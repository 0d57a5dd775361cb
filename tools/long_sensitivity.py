"""How sensitive is the reference's own closed loop to the QP solve accuracy?  (CPU, dev container)

Re-runs tests/golden/make_golden.py's gen_long_closed_loop (the reference's example/rqp_example.py
loop, imported behind tests/golden/refstubs.py, every QP answered by the oracle IPM) with the IPM
tolerance changed from the fixture's 1e-11 to `tol`, over `T` seconds, and reports where its f_des /
states leave 1e-5 / 1e-4 of the committed fixture -- i.e. the divergence onset between two solves of
the SAME reference loop that differ only in solver accuracy, to compare with the GPU's onset
(tests/test_gpu_long.py).

    python -O tools/long_sensitivity.py centralized 1e-12 35
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)

ct, tol, T = sys.argv[1], float(sys.argv[2]), float(sys.argv[3])
import oracle.ipm as oipm  # noqa: E402

_orig = oipm.solve_qp
oipm.solve_qp = lambda *a, **k: _orig(*a, **{**k, "tol": tol})
import make_golden as mg  # noqa: E402

mg.OUT = "/tmp"
mg.gen_long_closed_loop(ct, T=T)
tag = ct.split("-")[0][:4]
a = np.load(f"/tmp/ref_long_{tag}.npz")
b = np.load(os.path.join(ROOT, "tests", "golden", f"ref_long_{tag}.npz"))
K = a["f_des"].shape[0]
rel = np.array([np.max(np.abs(a["f_des"][k] - b["f_des"][k])) / max(1.0, np.max(np.abs(b["f_des"][k]))) for k in range(K)])
ds = np.max(np.abs(a["states"] - b["states"][: a["states"].shape[0]]), axis=1)
every = int(a["state_every"])
of = int(np.argmax(rel > 1e-5)) if np.any(rel > 1e-5) else None
os_ = int(np.argmax(ds > 1e-4)) * every if np.any(ds > 1e-4) else None
print(f"{ct}: IPM tol {tol:g} vs 1e-11 over {T:.0f} s: f_des leaves 1e-5 at HL step {of}, states leave 1e-4 at HL step "
      f"{os_}; max f_des rel diff {rel.max():.2e}")
