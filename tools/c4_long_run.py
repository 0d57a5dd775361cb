"""C4 over SURVEY 8(d)'s 10 s closed loop: 1,000 HL steps of the bench's default workload (65,536 path-start
scenarios in 64 seeded forests), reported per block of 100 steps -- ms per step (block mean, and the
p50 / p99 of the per-step clock marks), agent QPs, mean ADMM passes per scenario and step, IPM
iterations per agent QP, in-band exits (and beyond Clarabel's 1e-8), collisions.

    python tools/c4_long_run.py [steps] [block] [out.json]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_aerial_transportation_amd import BatchedController, scenarios  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
block = int(sys.argv[2]) if len(sys.argv) > 2 else 100
out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "gpurun_out", "c4_long_run.json")
n, B = 6, 65536
sf, st, forests = bench.bench_states(n, B, 0, 1, 64, "path", None)
eng = BatchedController("cadmm", n, B, scenarios.params_block(n))
eng.set_forests(forests, sf)
eng.set_state(st, np.zeros(B, dtype=np.int32))
subs = int(os.environ.get("SUBS", "1"))  # sub-batch streams (dat_set_sub_batches); marks then hold start / end only
if subs > 1:
    eng.set_sub_batches(subs)
rows = []
for b0 in range(0, steps, block):
    eng.reset_counters()
    eng.synchronize()
    t0 = time.perf_counter()
    eng.closed_loop(block)
    eng.synchronize()
    dt = time.perf_counter() - t0
    w = eng.work()
    per = np.diff(eng.step_marks())
    r = eng.control(None, None)  # metrics of the state after the block (one more HL step, not timed)
    eng.rollout(10)
    row = {"steps": [b0, b0 + block], "ms_per_step": dt / block * 1e3, "p50_ms": float(np.percentile(per, 50)),
           "p99_ms": float(np.percentile(per, 99)), "agent_qps": w["qp_solves"],
           "agent_qps_per_s": w["qp_solves"] / dt, "mean_admm_passes": w["qp_solves"] / (n * B * block),
           "ipm_iters_per_qp": w["ipm_iters"] / max(w["qp_solves"], 1), "inband_exits": w["inband_exits"],
           "inband_beyond_clarabel_tol": w["inband_beyond_clarabel_tol"],
           "collisions_after_block": int(r.collision.sum()), "min_env_dist_after_block": float(r.min_env_dist.min())}
    rows.append(row)
    print(json.dumps(row), flush=True)
os.makedirs(os.path.dirname(out), exist_ok=True)
with open(out, "w") as f:
    json.dump({"workload": "C4: cadmm n=6, forest env (path start), 65536 closed-loop scenarios, 1 GPU"
               + (f", {subs} sub-batch streams" if subs > 1 else ""), "blocks": rows}, f, indent=1)
