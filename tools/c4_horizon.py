"""Write tests/golden/c4_horizon.json from the reference's own C4 loop at two QP tolerances
(tests/golden/ref_c4_loop.npz at 1e-11 and the tools/c4_sensitivity.py re-run at 1e-10): per scenario,
the first HL step at which f_des leaves 1e-5 (relative), the ADMM iteration count differs, and the
state leaves 1e-4 (None: never within the recorded horizon).

    python tools/c4_horizon.py /tmp/ref_c4_loop.npz
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
a = np.load(os.path.join(ROOT, "tests", "golden", "ref_c4_loop.npz"))
b = np.load(sys.argv[1])
out = {"source": "reference loop (make_golden.gen_c4_loop) at oracle QP tol 1e-11 vs 1e-10 (tools/c4_sensitivity.py)"}
for s in range(len(a["seeds"])):
    fa, fb = a[f"s{s}_f_des"], b[f"s{s}_f_des"]
    K = min(len(fa), len(fb))
    df = np.array([np.max(np.abs(fa[k] - fb[k])) / max(1.0, np.max(np.abs(fa[k]))) for k in range(K)])
    di = a[f"s{s}_iters"][:K] != b[f"s{s}_iters"][:K]
    dx = np.max(np.abs(a[f"s{s}_states"][:K] - b[f"s{s}_states"][:K]), axis=1) > 1e-4
    first = lambda m: int(np.argmax(m)) if m.any() else None  # noqa: E731
    out[str(s)] = {"f": first(df > 1e-5), "iters": first(di), "state": first(dx)}
    print(s, out[str(s)], f"max f diff before onset {df[:out[str(s)]['f'] or K].max():.2e}")
with open(os.path.join(ROOT, "tests", "golden", "c4_horizon.json"), "w") as f:
    json.dump(out, f, indent=1)
