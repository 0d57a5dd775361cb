"""Per-call latency of the drop-in controllers (one scenario, B = 1) against the reference's 10 ms
high-level period (example/rqp_example.py:85-86: dt = 1e-3, hl_rel_freq = 10), on the GPU box.

    python tools/dropin_latency.py [steps]

For each controller: the reference's loop on the seed-0 forest (forest desired-acceleration law on the
host, ctl.control(state, acc) per HL step, 10 simulation steps on a separate GPU dynamics engine);
reports the wall time of control() per call (mean / p50 / p99 / max, ms) including the host-device
copies and synchronisation, the GPU kernel time inside it (SolverStatistics.solve_time) and the ADMM /
DD iteration counts.  Prints one JSON line."""

import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_aerial_transportation_amd as dat  # noqa: E402
from distributed_aerial_transportation_amd import BatchedController, Forest, example, scenarios, system  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    out = {"hl_period_ms": 10.0, "steps": steps}
    forest = Forest.seeded(0)
    for name in ("RQPCentralizedController", "RQPCADMMController", "RQPDDController"):
        p, col, s0 = scenarios.rqp_setup(3)
        ctl = getattr(dat, name)(p, col, s0, 1e-3, forest)
        sim = BatchedController("cadmm", 3, 1, system.pack_params(p, col))
        sim.set_state(system.pack_state(s0)[None], np.zeros(1, dtype=np.int32))
        wall, kern, its = [], [], []
        for k in range(steps):
            x, _ = sim.get_state()
            st = system.RQPState.unpack(x[0], 3)
            x_ref, v_ref = example.references(st.xl[None], forest)
            dvl = -(st.vl - v_ref[0]) - (st.xl - x_ref[0])
            nrm = np.linalg.norm(dvl)
            if nrm > 0:
                dvl = dvl / nrm * min(nrm, 1.0)
            t0 = time.perf_counter()
            f, stats = ctl.control(st, (dvl, np.zeros(3)))
            wall.append((time.perf_counter() - t0) * 1e3)
            kern.append(stats.solve_time * 1e3)
            its.append(stats.iter)
            sim.rollout(10, f[None])
        w = np.array(wall[5:])
        out[name] = {"wall_ms_mean": float(w.mean()), "wall_ms_p50": float(np.percentile(w, 50)),
                     "wall_ms_p99": float(np.percentile(w, 99)), "wall_ms_max": float(w.max()),
                     "gpu_ms_mean": float(np.mean(kern[5:])), "mean_iters": float(np.mean(its[5:])),
                     "max_iters": int(np.max(its[5:]))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
