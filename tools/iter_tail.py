"""Outer-iteration (ADMM / DD) distribution of a QP-level bench configuration (GPU): how long is the
tail of scenarios a persistent drain waits for, and does the previous step's count predict it?

    python tools/iter_tail.py --config C3|C2|C5
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_aerial_transportation_amd import BatchedController  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--steps", type=int, default=4)
args = ap.parse_args()
n, mode, B = bench.QP_CONFIGS[args.config]
rng = np.random.default_rng(2000)
states, accs, params, per = bench.qp_level_inputs(args.config, n, B, rng)
eng = BatchedController(mode, n, B, params, per_scenario_params=per)
its = []
for k in range(args.steps):
    r = eng.control(states if k == 0 else None, accs[k])
    its.append(np.asarray(r.iters).copy())
it = np.stack(its)
for k in range(args.steps):
    h = np.bincount(it[k])
    q = np.percentile(it[k], [50, 90, 99, 99.9, 100])
    print(f"{args.config} step {k}: mean {it[k].mean():.2f}, p50/p90/p99/p99.9/max {q}, "
          f"scenarios >= 2x mean {int((it[k] >= 2 * it[k].mean()).sum())}")
    print("   " + " ".join(f"{j}:{int(v)}" for j, v in enumerate(h) if v))
for k in range(1, args.steps):
    print(f"corr(step {k - 1}, step {k}) = {np.corrcoef(it[k - 1], it[k])[0, 1]:.3f}")
