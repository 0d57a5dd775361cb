"""Latency of one stalled C4 scenario alone on the GPU (a state captured by tools/c4_stall_states.py):
two HL steps (the second a 101-pass max_iter stall), device time per step and per IPM iteration.

    python tools/stall_latency.py states.npz [scenario] [steps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_aerial_transportation_amd import BatchedController, scenarios  # noqa: E402

d = np.load(sys.argv[1])
j = int(sys.argv[2]) if len(sys.argv) > 2 else 0
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
n = 6
forests = bench.bench_states(n, 1, 0, 1, 64, "path", None)[2]
eng = BatchedController("cadmm", n, 1, scenarios.params_block(n))
eng.set_forests(forests, d["scen_forest"][j:j + 1])
eng.set_state(d["states"][j:j + 1], np.zeros(1, dtype=np.int32))
for k in range(steps):
    w0, m0 = eng.work(), eng.kernel_ms()
    r = eng.control(None, None)
    eng.synchronize()
    w1, ms = eng.work(), eng.kernel_ms() - m0
    ipm = w1["ipm_iters"] - w0["ipm_iters"]
    print(f"step {k}: passes {int(r.iters[0])}, device {ms:.2f} ms, IPM iterations (all agents) {ipm}, "
          f"per pass {ms * 1e3 / max(int(r.iters[0]), 1):.1f} us", flush=True)
    eng.rollout(10)
