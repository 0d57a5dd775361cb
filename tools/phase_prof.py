"""IPM phase profile (GPU, development build): shader-clock cycles per ipm_solve phase summed over
wavefronts, for a build_var library compiled with -DDAT_PHASE_PROF.

    DAT_LIB_PATH=build_var/libdat_prof.so python tools/phase_prof.py [--config C4|C2|C3|C5]
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

NAMES = {0: "ipm init", 1: "residuals + stop test", 2: "NT scaling + D", 3: "M, chol, T, N, P", 4: "predictor newton",
         5: "affine step / gap / sigma", 6: "corrector newton (+refinement)", 7: "step, backtrack, update",
         8: "exit / best iterate", 9: "drain: after the solve (lane results)", 10: "(whole ipm_solve, drain's view)",
         11: "drain: slot refill + build_shared", 12: "drain: fresh slot: lane statics, env rows",
         13: "drain: consensus, dual update, outputs", 14: "drain: lane_cadmm_dynamic", 15: "drain: tuned flag, ipm call"}
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C4")
ap.add_argument("--steps", type=int, default=4)
args = ap.parse_args()
lib = L.lib()
lib.dat_get_phase_cycles.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 16)()
if args.config == "stall":  # the C4 stall stretches of ref_c4_hard.npz alone (the tail kernel's regime)
    from distributed_aerial_transportation_amd import Forest

    d = np.load(os.path.join(ROOT, "tests", "golden", "ref_c4_hard.npz"))
    n, J = 6, d["x0"].shape[0]
    eng = BatchedController("cadmm", n, J, scenarios.params_block(n))
    eng.set_forests([Forest.seeded(int(s)) for s in d["forest_seed"]], np.arange(J, dtype=np.int32))
    eng.set_state(d["x0"], np.zeros(J, dtype=np.int32))
    for k in range(2):
        eng.control(None, None)
        eng.rollout(10)
    lib.dat_get_phase_cycles(buf)
    for k in range(args.steps):
        eng.control(None, None)
        eng.rollout(10)
elif args.config == "C4":
    n, B = 6, 65536
    sf, st, forests = bench.bench_states(n, B, 0, 1, 64, "path", None)
    eng = BatchedController("cadmm", n, B, scenarios.params_block(n))
    eng.set_forests(forests, sf)
    eng.set_state(st, np.zeros(B, dtype=np.int32))
    eng.closed_loop(2)
    lib.dat_get_phase_cycles(buf)
    eng.closed_loop(args.steps)
else:
    n, mode, B = bench.QP_CONFIGS[args.config]
    rng = np.random.default_rng(2000)
    states, accs, params, per = bench.qp_level_inputs(args.config, n, B, rng)
    eng = BatchedController(mode, n, B, params, per_scenario_params=per)
    eng.set_state(states)
    for k in range(2):
        eng.control(None, L.f64(accs[k]))
    lib.dat_get_phase_cycles(buf)
    for k in range(args.steps):
        eng.control(None, L.f64(accs[2 + k]))
eng.synchronize()
lib.dat_get_phase_cycles(buf)
c = np.array(list(buf), dtype=np.float64)
tot = c.sum()
w = eng.work()
print(f"{args.config}: {args.steps} steps, {w['ipm_iters']} IPM iterations, {w['qp_solves']} QPs")
ipm = c[10]
print(f"  IPM {100 * ipm / (tot - sum(c[:9])):.1f} % of the drain's time; IPM phases as % of the whole:")
tot = tot - sum(c[:9])  # the ipm phases are inside phase 10
for k, name in NAMES.items():
    if c[k]:
        print(f"  {name:34s} {100 * c[k] / tot:5.1f} %   {c[k] / max(w['ipm_iters'], 1):9.0f} cycles per lane-iteration (wave sum)")
