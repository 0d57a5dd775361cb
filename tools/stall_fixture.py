"""Latency of the C4 stall stretches (tests/golden/ref_c4_hard.npz) on the GPU, each scenario alone (one
wavefront): per HL step the ADMM passes, the device time of the C-ADMM drain (k_cadmm + its hand-over
kernel), IPM iterations, in-band exits and hand-overs, and the time per pass and per critical-path IPM
iteration.  The stretches are the SURVEY's 10 s C4 loop's late regime (every step after the first a 101-pass
stall), so this is the step time a wedged scenario sets there.

    python tools/stall_fixture.py [json_out]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_aerial_transportation_amd import BatchedController, Forest, scenarios  # noqa: E402

d = np.load(os.path.join(ROOT, "tests", "golden", "ref_c4_hard.npz"))
n = 6
J, K = d["f_des"].shape[:2]
out = {"steps": []}
for j in range(J):
    eng = BatchedController("cadmm", n, 1, scenarios.params_block(n))
    eng.set_forests([Forest.seeded(int(d["forest_seed"][j]))], np.zeros(1, dtype=np.int32))
    eng.set_state(d["x0"][j:j + 1], np.zeros(1, dtype=np.int32))
    tot_ms = tot_pass = 0.0
    for k in range(K):
        eng.reset_counters()
        r = eng.control(None, None)
        eng.synchronize()
        w, ms = eng.work(), eng.kernel_ms()
        p = int(r.iters[0])
        ref = d["f_des"][j, k]
        rel = float(np.max(np.abs(r.f_des[0] - ref)) / max(1.0, np.max(np.abs(ref))))
        row = {"scenario": j, "step": k, "passes": p, "drain_ms": ms, "us_per_pass": ms * 1e3 / max(p, 1),
               "ipm_iters": w["ipm_iters"], "qp_solves": w["qp_solves"],
               "ipm_per_qp": w["ipm_iters"] / max(w["qp_solves"], 1), "inband": w["inband_exits"],
               "loose": w["inband_beyond_clarabel_tol"], "handovers": w["robust_redos"], "f_des_rel": rel,
               "iters_ref": int(d["iters"][j, k]), "tail_passes": w.get("tail_passes"),
               "tail_crit_ipm": w.get("tail_critical_ipm_iters"), "routed": w.get("tail_routed"),
               "certified": w.get("certified_infeasible"), "stall_exits": w.get("stall_exits"),
               "warm": w.get("warm_starts"), "refine_passes": w.get("refine_passes"),
               "refine_corrections": w.get("refine_corrections")}
        if k > 0:
            tot_ms += ms
            tot_pass += p
        out["steps"].append(row)
        print(json.dumps(row), flush=True)
        eng.rollout(10)
    eng.close()
    print(f"scenario {j}: stalled steps 1-{K - 1}: {tot_ms / (K - 1):.2f} ms per step, "
          f"{tot_ms * 1e3 / max(tot_pass, 1):.1f} us per pass", flush=True)
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as f:
        json.dump(out, f)
