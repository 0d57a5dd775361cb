"""Capture the states of the scenarios that stall longest in the C4 10 s loop (from
tools/c4_stall_probe.py's npz) one HL step before their first stall, then run those states alone on a
small handle: ADMM passes, IPM iterations per agent QP, statuses and step time.  Saves the states for a
CPU replay with the oracle.

    python tools/c4_stall_states.py probe.npz [count] [out.npz]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_aerial_transportation_amd import BatchedController, scenarios  # noqa: E402

probe = np.load(sys.argv[1])
count = int(sys.argv[2]) if len(sys.argv) > 2 else 12
out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "gpurun_out", "c4_stall_states.npz")
stalled, first = probe["stalled"], probe["first_stall"]
idx = np.argsort(-stalled)[:count]
cap = first[idx] - 1
n, B = 6, 65536
sf, st, forests = bench.bench_states(n, B, 0, 1, 64, "path", None)
eng = BatchedController("cadmm", n, B, scenarios.params_block(n))
eng.set_forests(forests, sf)
eng.set_state(st, np.zeros(B, dtype=np.int32))
S = st.shape[1]
states = np.zeros((count, S))
done = 0
for k in sorted(set(cap.tolist())):
    if k > done:
        eng.closed_loop(k - done)
        done = k
    x, _ = eng.get_state()
    for j in np.nonzero(cap == k)[0]:
        states[j] = x[idx[j]]
print("captured", count, "states at steps", cap.tolist(), flush=True)
sub = BatchedController("cadmm", n, count, scenarios.params_block(n), record_err=True)
sub.set_forests(forests, sf[idx])
sub.set_state(states, np.zeros(count, dtype=np.int32))
rows = []
for k in range(4):
    w0 = sub.work()
    t0 = time.perf_counter()
    r = sub.control(None, None)
    sub.synchronize()
    dt = (time.perf_counter() - t0) * 1e3
    w1 = sub.work()
    q = w1["qp_solves"] - w0["qp_solves"]
    ipm = w1["ipm_iters"] - w0["ipm_iters"]
    bad = (r.qp_status != 0).sum(axis=1) if r.qp_status.ndim > 1 else (r.qp_status != 0)
    print(f"step {k}: {dt:.1f} ms, ADMM passes {r.iters.tolist()}, IPM it/QP {ipm / max(q, 1):.2f}, "
          f"non-optimal agent QPs per scenario {np.asarray(bad).tolist()}, min env dist "
          f"{np.round(r.min_env_dist, 3).tolist()}", flush=True)
    rows.append(r.iters.copy())
    sub.rollout(10)
np.savez_compressed(out, idx=idx, cap=cap, states=states, scen_forest=sf[idx], iters=np.array(rows))
