"""Is a QP-level configuration's step time set by its slowest scenario?  Times the bench step (GPU)
with the outer-iteration cap lowered (set_max_iter): if the step time falls in proportion to the cap
while the mean iteration count barely moves, the step is the critical path of the scenarios that run
to the cap, not the throughput of the batch.

    python tools/critical_path.py --config C3|C2|C5
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_aerial_transportation_amd import BatchedController  # noqa: E402
from distributed_aerial_transportation_amd import _lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--steps", type=int, default=6)
args = ap.parse_args()
n, mode, B = bench.QP_CONFIGS[args.config]
for cap in (100, 50, 25, 12):
    rng = np.random.default_rng(2000)
    states, accs, params, per = bench.qp_level_inputs(args.config, n, B, rng)
    eng = BatchedController(mode, n, B, params, per_scenario_params=per)
    eng.set_max_iter(cap)
    eng.set_state(states)
    accs = [L.f64(a) for a in accs]
    lib, h = eng._lib, eng._h
    for k in range(2):
        L.check(lib.dat_control_step(h, None, L.ptr(accs[k]), None, None, None, None, None, None))
    eng.synchronize()
    its = []
    t0 = time.perf_counter()
    for k in range(args.steps):
        r = eng.control(None, accs[(2 + k) % len(accs)])
        its.append(np.asarray(r.iters))
    eng.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    it = np.concatenate(its)
    print(f"{args.config} max_iter {cap:3d}: {ms:7.2f} ms/step (incl. host copies), mean outer iterations "
          f"{it.mean():.2f}, at the cap {(it > cap).mean() * 100:.3f} % of scenarios")
