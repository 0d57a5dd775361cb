"""Diagnostics for tests/test_gpu_long.py: run example.simulate_batch on the GPU over `T` seconds and
save per-HL-step f_des, iters, min_dist and the state at every HL step (gpurun_out/long_<tag>.npz)."""
import sys

import numpy as np

sys.path.insert(0, ".")
from distributed_aerial_transportation_amd import BatchedController, Forest, scenarios, system  # noqa: E402

ct, T = sys.argv[1], float(sys.argv[2])
_, _, s0 = scenarios.rqp_setup(3)
eng = BatchedController(ct, 3, 1, scenarios.params_block(3))
eng.set_forests([Forest.seeded(0)])
eng.set_state(system.pack_state(s0)[None], np.zeros(1, dtype=np.int32))
F, I, MD, X, QS = [], [], [], [], []
for k in range(int(round(T / 1e-2))):
    x, _ = eng.get_state()
    X.append(x[0].copy())
    r = eng.control(None, None)
    F.append(r.f_des[0].copy()), I.append(r.iters[0]), MD.append(r.min_env_dist[0]), QS.append(r.qp_status[0].copy())
    if k % 1000 == 0:
        print(k, flush=True)
        np.savez(f"gpurun_out/long_{ct.split('-')[0][:4]}.npz", f_des=np.array(F), iters=np.array(I), min_dist=np.array(MD),
                 states=np.array(X), qp_status=np.array(QS))
    eng.rollout(10)
tag = ct.split("-")[0][:4]
np.savez(f"gpurun_out/long_{tag}.npz", f_des=np.array(F), iters=np.array(I), min_dist=np.array(MD), states=np.array(X), qp_status=np.array(QS))
print("saved", len(F))
