"""IPM iteration histogram of the agent QPs of a bench configuration (GPU, development build with
-DDAT_ITER_HIST): how wide is the spread a wavefront's pass waits for?

    DAT_LIB_PATH=build_var/libdat_hist.so python tools/iter_hist.py --config C3|C4|C2|C5
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_aerial_transportation_amd import BatchedController, scenarios  # noqa: E402
from distributed_aerial_transportation_amd import _lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--steps", type=int, default=4)
args = ap.parse_args()
lib = L.lib()
lib.dat_get_iter_hist.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 64)()
if args.config == "C4":
    n, B = 6, 65536
    sf, st, forests = bench.bench_states(n, B, 0, 1, 64, "path", None)
    eng = BatchedController("cadmm", n, B, scenarios.params_block(n))
    eng.set_forests(forests, sf)
    eng.set_state(st, np.zeros(B, dtype=np.int32))
    eng.closed_loop(2)
    lib.dat_get_iter_hist(buf)
    eng.closed_loop(args.steps)
else:
    n, mode, B = bench.QP_CONFIGS[args.config]
    rng = np.random.default_rng(2000)
    states, accs, params, per = bench.qp_level_inputs(args.config, n, B, rng)
    eng = BatchedController(mode, n, B, params, per_scenario_params=per)
    eng.set_state(states)
    for k in range(2):
        eng.control(None, L.f64(accs[k]))
    lib.dat_get_iter_hist(buf)
    for k in range(args.steps):
        eng.control(None, L.f64(accs[2 + k]))
eng.synchronize()
lib.dat_get_iter_hist(buf)
h = np.array(list(buf), dtype=np.float64)
tot = h.sum()
mean = (h * np.arange(64)).sum() / tot
cdf = np.cumsum(h) / tot
q = {p: int(np.searchsorted(cdf, p)) for p in (0.5, 0.9, 0.99, 0.999)}
# expected maximum over a wavefront of 60 independent solves
emax = sum(1.0 - cdf[k] ** 60 for k in range(63))
print(f"{args.config}: {int(tot)} agent QPs, mean {mean:.2f} IPM iterations, quantiles {q}, "
      f"E[max of 60] {emax:.1f} -> ideal lane utilisation {mean / emax:.2f}")
print("  " + " ".join(f"{k}:{int(v)}" for k, v in enumerate(h) if v))
