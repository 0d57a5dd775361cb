"""Where the C4 10 s loop spends its time: per HL step of the bench's default workload, the ADMM
iteration distribution (scenarios at max_iter + 1 = 101 passes, > 30, > 10), the wall time, collisions,
and per scenario the number of stalled steps (iters > 100) -- are stalls transient or persistent?

    python tools/c4_stall_probe.py [steps] [out.npz]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_aerial_transportation_amd import BatchedController, scenarios  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "c4_stall_probe.npz")
n, B = 6, 65536
sf, st, forests = bench.bench_states(n, B, 0, 1, 64, "path", None)
eng = BatchedController("cadmm", n, B, scenarios.params_block(n))
eng.set_forests(forests, sf)
eng.set_state(st, np.zeros(B, dtype=np.int32))
stalled = np.zeros(B, dtype=np.int32)
first = np.full(B, -1, dtype=np.int32)
rows = []
for k in range(steps):
    t0 = time.perf_counter()
    r = eng.control(None, None)
    eng.rollout(10)
    eng.synchronize()
    dt = (time.perf_counter() - t0) * 1e3
    it = r.iters
    s = it > 100
    stalled += s
    first[(first < 0) & s] = k
    rows.append((k, dt, int(s.sum()), int((it > 30).sum()), int((it > 10).sum()), float(it.mean()),
                 int(r.collision.sum()), float(r.min_env_dist.min()), int((r.qp_status != 0).sum())))
    if k % 50 == 0:
        print(rows[-1], flush=True)
np.savez_compressed(out, steps=np.array(rows), stalled=stalled, first_stall=first, scen_forest=sf)
ever = stalled > 0
print("scenarios that ever stall:", int(ever.sum()), "stalled steps per such scenario: mean",
      float(stalled[ever].mean()) if ever.any() else 0, "max", int(stalled.max()))
