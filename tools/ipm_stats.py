"""Corrector refinement statistics of the agent QPs on the C4 closed loop (CPU, host build of the same
per-lane code with -DDAT_IPM_STATS): corrector solves, refinement passes run, passes stopped by the
rounding-level test.

    python tools/ipm_stats.py [scenarios] [hl_steps]
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import cpu_baseline as cb  # noqa: E402
from distributed_aerial_transportation_amd import scenarios  # noqa: E402

LIB = "/tmp/libdat_cpu_stats.so"
subprocess.check_call(["hipcc", "-O3", "-march=x86-64-v3", "-fopenmp", "-std=c++17", "-fPIC", "-shared", "-DDAT_IPM_STATS",
                       "--offload-arch=gfx950", cb.SRC, "-o", LIB])
cb.LIB = LIB
L = cb.lib()
L.datcpu_ipm_stats.argtypes = [ctypes.POINTER(ctypes.c_longlong)]
S = int(sys.argv[1]) if len(sys.argv) > 1 else 512
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
n = 6
sf, st, forests = bench.bench_states(n, S, 0, 1, 64, "path", None)
c = cb.CpuClosedLoop(n, S, scenarios.params_block(n))
c.set_forests(forests, sf)
c.set_state(st)
c.closed_loop(2, threads=1)
buf = (ctypes.c_longlong * 88)()
L.datcpu_ipm_stats(buf)
q, it = c.closed_loop(K, threads=1)
L.datcpu_ipm_stats(buf)
corr, passes, early = buf[0], buf[1], buf[2]
print(f"{q} agent QPs, {it} IPM iterations ({it / q:.2f}/QP); corrector solves {corr}; refinement passes run "
      f"{passes} ({passes / max(corr, 1):.2f} per corrector), of which stopped at the rounding test {early}; "
      f"refinement corrections applied {passes - early} ({(passes - early) / max(corr, 1):.2f} per corrector)")
print("non-converged IPM exits by reason (1 non-finite, 2 divergence / max_iter, 3 cone scaling, 4 cone block D, "
      f"5 Cholesky of M, 6 Cholesky of N): {list(buf[4:10])}")
h = np.array(list(buf)[16:]).reshape(3, 24)
print("log10(max row z/s) bin: [first refinement pass stopped at rounding, correction applied, second pass run]")
for b in range(24):
    if h[:, b].any():
        print(f"  1e{b - 12:+d}: {h[0, b]:8d} {h[1, b]:8d} {h[2, b]:8d}")
L.datcpu_ipm_ith.argtypes = [ctypes.POINTER(ctypes.c_longlong)]
ith = (ctypes.c_longlong * 512)()
L.datcpu_ipm_ith(ith)
c.closed_loop(K, threads=1)
L.datcpu_ipm_ith(ith)
H = np.array(list(ith)).reshape(2, 8, 32)
print(f"IPM iterations by start (tuned / conservative) and active env rows ({K} more HL steps):")
for t in (1, 0):
    for e in range(8):
        row = H[t, e]
        if row.sum():
            mean = (row * np.arange(32)).sum() / row.sum()
            print(f"  {'tuned' if t else 'cons.'} env rows {e}: {int(row.sum()):7d} QPs, mean {mean:.2f}: "
                  + " ".join(f"{k}:{int(v)}" for k, v in enumerate(row) if v))
