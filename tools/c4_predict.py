"""C4 (GPU): which per-scenario quantities known before a control step predict its ADMM iteration
count -- the previous step's count, the env class / min env distance of this step's state?"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_aerial_transportation_amd import BatchedController, scenarios  # noqa: E402

n, B = 6, int(os.environ.get("B", 65536))
sf, states, forests = bench.bench_states(n, B, 0, 1, 64, "path", None)
eng = BatchedController("cadmm", n, B, scenarios.params_block(n))
eng.set_forests(forests, sf)
eng.set_state(states, np.zeros(B, dtype=np.int32))
prev = None
rows = []
for k in range(int(os.environ.get("STEPS", 14))):
    lhs, rhs, nr, col, md = eng.env_rows()       # this step's env rows (state before control)
    r = eng.control(None, None)
    if k >= 2:
        rows.append(np.stack([prev, r.iters, nr.max(axis=1), md.min(axis=1), r.min_env_dist], 1))
    prev = r.iters.copy()
    eng.rollout(10)
a = np.concatenate(rows)
p_it, it, nrow, mdist = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
long_ = it >= 8
print(f"samples {len(a)}, long (>= 8 ADMM iters): {int(long_.sum())}")
for name, v, thr in (("prev iters >= 4", p_it, 4), ("prev iters >= 6", p_it, 6), ("env rows >= 3", nrow, 3),
                     ("env rows >= 5", nrow, 5), ("min env dist < 1.0", -mdist, -1.0), ("min env dist < 0.5", -mdist, -0.5)):
    sel = v >= thr
    print(f"{name:22s}: selects {int(sel.sum()):6d} ({sel.mean() * 100:5.2f} %), recall of long {np.sum(sel & long_) / max(long_.sum(), 1):.2f}")
for lo, hi in ((0, 0.3), (0.3, 0.6), (0.6, 1.0), (1.0, 2.0), (2.0, 99)):
    sel = (mdist >= lo) & (mdist < hi)
    if sel.any():
        print(f"min dist [{lo}, {hi}): n {int(sel.sum()):6d}  mean iters {it[sel].mean():.2f}  p99 {np.percentile(it[sel], 99):.0f}  "
              f"max {it[sel].max():.0f}")
for pv in range(1, 8):
    sel = p_it == pv
    if sel.any():
        print(f"prev iters {pv}: n {int(sel.sum()):6d}  mean {it[sel].mean():.2f}  p99 {np.percentile(it[sel], 99):.0f}  max {it[sel].max():.0f}")
