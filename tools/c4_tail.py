"""C4 tail diagnostic (GPU): per HL step, the distribution of ADMM iterations over the 65,536 scenarios
and the step's k_cadmm time, then the k_cadmm time of a batch made of only the step's slowest
scenarios (their own states and warm state replayed on a fresh handle) -- is a step's time set by
throughput or by the serial ADMM chain of its slowest scenario?"""
import os
import sys
import time

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
for k in range(int(os.environ.get("STEPS", 12))):
    x, cnt = eng.get_state()
    eng.reset_counters()
    r = eng.control(None, None)
    ms = eng.kernel_ms()
    it = r.iters
    q = np.percentile(it, [50, 99, 99.9, 100])
    print(f"step {k:2d}: k_cadmm {ms:6.3f} ms  ADMM iters p50 {q[0]:.0f} p99 {q[1]:.0f} p99.9 {q[2]:.0f} max {q[3]:.0f}  "
          f"#>=10: {int(np.sum(it >= 10))}  #>=20: {int(np.sum(it >= 20))}", flush=True)
    eng.rollout(10)
# the slowest scenarios of the last step alone (fresh warm state: the solo chain length)
idx = np.argsort(-it)[:64]
solo = BatchedController("cadmm", n, 64, scenarios.params_block(n))
solo.set_forests(forests, sf[idx])
solo.set_state(x[idx], cnt[idx])
solo.reset_counters()
r2 = solo.control(None, None)
print(f"64 slowest alone (fresh warm state): k_cadmm {solo.kernel_ms():.3f} ms, iters {sorted(r2.iters.tolist())[-8:]}")
one = BatchedController("cadmm", n, 1, scenarios.params_block(n))
one.set_forests(forests, sf[idx[:1]])
one.set_state(x[idx[:1]], cnt[idx[:1]])
one.reset_counters()
r3 = one.control(None, None)
w = one.work()
print(f"slowest alone: k_cadmm {one.kernel_ms():.3f} ms, ADMM iters {r3.iters[0]}, IPM iters {w['ipm_iters']} over {w['qp_solves']} QPs")
