"""Run rqp_example's 100 s closed loop (n = 3, forest seed 0) on the GPU as tests/test_gpu_long.py does and save
the logs (f_des, ADMM iterations, min env distance per HL step; the packed state per log step) for a CPU replay
of the states past the reference's reproducibility horizon.

    python tools/long_dump.py consensus-admm|dual-decomposition|centralized [out.npz]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_aerial_transportation_amd import Forest, example, scenarios, system  # noqa: E402

ct = sys.argv[1] if len(sys.argv) > 1 else "consensus-admm"
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", f"long_{ct}.npz")
_, _, s0 = scenarios.rqp_setup(3)
logs = example.simulate_batch(ct, system.pack_state(s0)[None], [Forest.seeded(0)], n=3, T=100.0, progress=True)[0]
md = np.array(logs["min_env_dist_seq"])
np.savez_compressed(out, f_des=np.array(logs["f_des_seq"]), iters=np.array(logs["iter_seq"]), min_dist=md,
                    states=np.array([system.pack_state(s) for s in logs["state_seq"]]))
print(f"{ct}: min env dist {md.min():.4f} at HL step {int(np.argmin(md))}; collisions (HL steps with dist < 0) "
      f"{int((md < 0).sum())}, first at {int(np.argmax(md < 0)) if np.any(md < 0) else None}")
