"""Capture the agent QPs the tail accepts in band beyond Clarabel's 1e-8 over SURVEY 8(d)'s 10 s C4 loop (a
-DDAT_CAPTURE_LOOSE build, tools/build_var.sh loose -DDAT_CAPTURE_LOOSE; run with DAT_LIB_PATH pointing at it):
their inputs -- scenario state, acc_des, agent, the pass's multipliers, mean and rho, the forest -- to
tests/golden/loose_caps.npz, answered by the oracle in tests/golden/make_loose_caps.py.

    DAT_LIB_PATH=build_var/libdat_loose.so python tools/capture_loose.py [steps] [out.npz]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_aerial_transportation_amd import BatchedController, scenarios  # noqa: E402
from distributed_aerial_transportation_amd import _lib as L  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "loose_caps.npz")
n, B = 6, 65536
sf, st, forests = bench.bench_states(n, B, 0, 1, 64, "path", None)
eng = BatchedController("cadmm", n, B, scenarios.params_block(n))
eng.set_forests(forests, sf)
eng.set_state(st, np.zeros(B, dtype=np.int32))
for b0 in range(0, steps, 100):
    eng.closed_loop(min(100, steps - b0))
    w = eng.work()
    print(f"steps {b0}-{b0 + 99}: loose {w['inband_beyond_clarabel_tol']}", flush=True)
cap = np.zeros((64, 320))
cnt = ctypes.c_int()
lib = L.lib()
lib.dat_get_captures.argtypes = [L.D, ctypes.POINTER(ctypes.c_int)]
L.check(lib.dat_get_captures(L.ptr(cap), ctypes.byref(cnt)))
k = min(cnt.value, 64)
S, N3 = st.shape[1], 3 * n
c = cap[:k]
np.savez(out, scenario=c[:, 0].astype(int), agent=c[:, 1].astype(int), admm_pass=c[:, 2].astype(int), rho=c[:, 3],
         prev_iters=c[:, 4].astype(int), forest=c[:, 5].astype(int), merit=c[:, 6], acc=c[:, 8:14],
         state=c[:, 14:14 + S], lam=c[:, 14 + S:14 + S + N3], fbar=c[:, 14 + S + N3:14 + S + 2 * N3])
print(f"captured {cnt.value} loose accepts ({k} kept) -> {out}; merits {np.round(c[:, 6], 10).tolist()}")
