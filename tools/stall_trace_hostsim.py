"""Per-iteration merit traces of the C4 stall stretches' agent QPs on the host build of the device solver
(TEST-infrastructure replay, as tests/test_hostsim.py::test_c4_stall_stretch_matches_oracle runs it), for
the design of the IPM's stall exit: for every agent QP, its IPM iterations, how it ended, and the iteration
at which its Clarabel-measured merit first fell below 1e-8 and reached its minimum.

    hipcc -O2 -std=c++17 -fPIC -shared --offload-arch=gfx950 -DDAT_IPM_TRACE tests/hostsim/hostsim.hip -o /tmp/hs_trace.so
    python tools/stall_trace_hostsim.py /tmp/hs_trace.so [steps] [out.json]
"""
import ctypes
import json
import os
import re
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests import hostsim as hs  # noqa: E402
from tests._golden import load  # noqa: E402

hs.LIB = sys.argv[1]
hs.build = lambda force=False: hs.LIB  # noqa: E731  (prebuilt variant)
K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
libc = ctypes.CDLL(None)

from distributed_aerial_transportation_amd import scenarios  # noqa: E402
from distributed_aerial_transportation_amd.system import RQPState, pack_state  # noqa: E402
from oracle import controllers as oc  # noqa: E402
from oracle import forest as of  # noqa: E402
from oracle import model as om  # noqa: E402
from oracle import scenarios as osc  # noqa: E402

LINE = re.compile(r"ipm it\s+(\d+) pres (\S+) dres (\S+) gap (\S+) merit (\S+) pobj (\S+)")
tmp = tempfile.NamedTemporaryFile(delete=False, suffix=".trace")
fd_save = os.dup(1)
os.dup2(tmp.fileno(), 1)


def mark(s):
    libc.fflush(None)
    os.write(1, (s + "\n").encode())


d = load("ref_c4_hard.npz")
n = 6
p = osc.params(n)
prm = scenarios.params_block(n)
for j in range(d["x0"].shape[0]):
    np.random.seed(int(d["forest_seed"][j]))
    forest = of.Forest()
    s0 = RQPState.unpack(d["x0"][j], n)
    st = om.State(s0.R, s0.w, s0.xl, s0.vl, s0.Rl, s0.wl, project=False)
    ctl = oc.CADMM(p, osc.col_radius(n), forest)
    tally = {"pass": 0, "tuned": 1, "step": 0}

    def solve(self, i, s_, acc, env, rho):
        lam = self.lam[:, :, i].T.reshape(-1).copy()
        fbar = self.f_mean.T.reshape(-1).copy()
        tuned = tally["tuned"] if tally["pass"] == 0 else 0
        f, status, its, inb = hs.qp_cadmm_ex(prm, n, pack_state(s_), np.concatenate(acc), env.lhs, env.rhs, i, lam,
                                             fbar, rho, tuned=tuned)
        m, ib, why = hs.last_diag()
        mark(f"SOLVE {j} {tally['step']} {tally['pass']} {i} {status} {its} {ib} {why} {m:.3e} {len(env.rhs)}")
        if status == 0:
            self.prev_f[i] = f.reshape(n, 3).T.copy()
        if i == n - 1:
            tally["pass"] += 1
        return self.prev_f[i], None

    ctl.solve_agent = solve.__get__(ctl)
    prev = 0
    for k in range(K):
        tally["pass"], tally["tuned"], tally["step"] = 0, 1 if prev <= 3 else 0, k
        acc, _, _ = oc.desired_acceleration_forest(st, forest)
        f, stat = ctl.control(st, acc)
        prev = stat.iter
        ref = d["f_des"][j, k]
        rel = np.max(np.abs(f - ref)) / max(1.0, np.max(np.abs(ref)))
        mark(f"STEP {j} {k} {stat.iter} {rel:.3e}")
        for _ in range(10):
            fl, M = om.low_level_control(p, st, f)
            st.integrate(*om.forward_dynamics(p, st, fl, M), 1e-3)
libc.fflush(None)
os.dup2(fd_save, 1)

# parse: the "ipm it" lines before a SOLVE marker belong to that solve (all of its attempts)
solves, steps, cur = [], [], []
for line in open(tmp.name):
    m = LINE.search(line)
    if m:
        it, pres, dres, grel, merit, pobj = m.groups()
        pres, dres, grel, pobj = float(pres), float(dres), float(grel), float(pobj)
        gap = grel * max(1.0, 0.01 * abs(pobj))
        mclr = max(pres, dres, gap / max(1.0, abs(pobj)))
        cur.append((int(it), float(merit), mclr))
    elif line.startswith("SOLVE"):
        t = line.split()
        solves.append({"scen": int(t[1]), "step": int(t[2]), "pass": int(t[3]), "agent": int(t[4]), "status": int(t[5]),
                       "iters": int(t[6]), "inband": int(t[7]), "why": int(t[8]), "merit": float(t[9]), "nenv": int(t[10]),
                       "trace": cur})
        cur = []
    elif line.startswith("STEP"):
        t = line.split()
        steps.append({"scen": int(t[1]), "step": int(t[2]), "iters": int(t[3]), "rel": float(t[4])})
os.unlink(tmp.name)

# critical path: per (scenario, step, pass) the max over agents of the IPM iterations
cp = {}
for s in solves:
    key = (s["scen"], s["step"])
    cp.setdefault(key, {}).setdefault(s["pass"], []).append(s["iters"])
for st_ in steps:
    key = (st_["scen"], st_["step"])
    passes = cp.get(key, {})
    crit = sum(max(v) for v in passes.values())
    tot = sum(sum(v) for v in passes.values())
    print(f"scen {key[0]} step {key[1]:2d}: passes {st_['iters']:3d} f_des rel {st_['rel']:.2e} critical-path IPM "
          f"iterations {crit:5d} (per pass {crit / max(len(passes), 1):.1f}), all {tot}")
ib = [s for s in solves if s["inband"]]
print(f"solves {len(solves)}, in-band exits {len(ib)}, iterations of in-band exits: mean "
      f"{np.mean([s['iters'] for s in ib]) if ib else 0:.1f}")
# first attempt's trace: iteration where mclr < 1e-8 first and where it is minimal
first_ok, at_min = [], []
for s in ib:
    tr = s["trace"]
    ok = [t for t in tr if t[2] < 1e-8]
    if ok:
        first_ok.append(tr.index(ok[0]))
        at_min.append(int(np.argmin([t[2] for t in tr])))
if first_ok:
    print(f"in-band exits: trace index of first mclr < 1e-8: mean {np.mean(first_ok):.1f}, of min mclr: mean "
          f"{np.mean(at_min):.1f}; trace length mean {np.mean([len(s['trace']) for s in ib]):.1f}")
if len(sys.argv) > 3:
    with open(sys.argv[3], "w") as f:
        json.dump({"solves": solves, "steps": steps}, f)
