"""Benchmark: agent-QP solves/s (node) + ms per control step, 6-quadrotor C-ADMM (BASELINE.json).

Workload (per GPU): n = 6 C-ADMM in the forest environment, B = 65536
closed-loop scenarios per GPU (weak scaling), 64 seeded forests (scenario s uses forest s mod 64),
start xl = (U(-2,0), U(-10,10), 1.5), vl = (0.5, 0, 0).  One "step" = one high-level period of
every scenario, fully on device: forest desired-acceleration law + C-ADMM control step (env CBF
rows, up to 101 ADMM iterations of n agent QPs each) + 10 simulation steps (SO(3) PD + dynamics).

    python bench.py [--gpus N --steps K --warmup W --batch B --n 6 --mode cadmm]
    python bench.py --gpus N   (default: strong scaling, BASELINE configs[3]: 65,536 scenarios split over
                                the N GPUs, the same global scenario set for every N)
    python bench.py --gpus N --batch 65536   (weak scaling: 65,536 scenarios per GPU)
    python bench.py --config C2|C3|C5 [--fixed-work]   (QP-level configs of SURVEY.md 8(d))
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

The data path has no collective; RCCL over xGMI (sharding.Comm, libdat.so's dat_comm_* C-ABI: no PyTorch in
the rank processes) carries the barrier, the max-over-ranks time and an all-gather of the per-scenario metrics.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6      # MI355X FP64 vector peak (AMD spec)
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md
# Algorithmic FP64 flops of the executed IPM work, counted per stage of the reduced
# agent QP: per IPM iteration BASE + ROW x R (R = active constraint rows; residuals, NT scalings, the
# u-space factorisations, the predictor and corrector solves without refinement, step lengths and the
# update), per refinement pass run PASS + PASS_ROW x R (the residual of the linearised system), per
# correction applied CORR (a core solve).  The kernels count IPM iterations, iterations x rows,
# refinement passes and corrections on device (dat_get_counters, dat_get_refinement_counters).
# Centralized (one cone block per lane, u-space algebra counted once per QP): per-block and u-space
# parts of the same stages, BASE = 1342 + 2027 n, PASS = 132 + 165 n, CORR = 72 + 180 n.
FLOP_MODEL = {
    "cadmm": dict(base=3975.0, row=215.0, ref=337.0, ref_row=17.0, corr=486.0),
    "dd": dict(base=2614.0, row=215.0, ref=207.0, ref_row=17.0, corr=150.0),
    "centralized": dict(base=1342.0, base_n=2027.0, row=215.0, ref=132.0, ref_n=165.0, ref_row=17.0, corr=72.0,
                        corr_n=180.0),
}


def model_flops(mode: str, n: int, ipm: float, rowit: float, refs: float, corrs: float) -> float:
    """Executed algorithmic flops (FLOP_MODEL) from the device work counters."""
    m = FLOP_MODEL[mode]
    rbar = rowit / max(ipm, 1.0)
    return ((m["base"] + m.get("base_n", 0.0) * n) * ipm + m["row"] * rowit
            + (m["ref"] + m.get("ref_n", 0.0) * n + m["ref_row"] * rbar) * refs + (m["corr"] + m.get("corr_n", 0.0) * n) * corrs)


def model_string(mode: str) -> str:
    m = FLOP_MODEL[mode]
    nb = lambda k: f" + {m[k + '_n']:.0f} n" if k + "_n" in m else ""  # noqa: E731
    return (f"per IPM iteration {m['base']:.0f}{nb('base')} + {m['row']:.0f} x active rows; per refinement pass "
            f"{m['ref']:.0f}{nb('ref')} + {m['ref_row']:.0f} x rows; per correction {m['corr']:.0f}{nb('corr')}")


TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


def traffic_per_launch(kernel: str, workload: str):
    """HBM bytes per launch of `kernel` from the committed PMC summary (tools/summarize_prof.py),
    if it was taken on this workload; None otherwise."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None
    e = t.get(kernel)
    if not e or e.get("workload") != workload:
        return None, None
    return e["bytes_per_launch"], e.get("source")


def auto_sub_batches(per_gpu: int) -> int:
    """C4 stream count per GPU.  A drain of 65,536 scenarios fills the chip and its tail is short (4 streams:
    3.73 -> 3.49 ms per step, +6 %, and the per-launch roofline would then split over 4 concurrent launches);
    at the per-GPU batches of the 2-, 4- and 8-GPU splits the slowest scenarios' passes dominate each step
    and 4 streams overlap one sub-batch's tail with the others' work: 32,768 3.06 -> 2.69, 16,384
    2.62 -> 2.20, 8,192 2.24 -> 1.82 ms per step (round 4 A/B, tools/r04_subs.sh)."""
    return 1 if per_gpu >= 65536 else 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None,
                    help="weak scaling: this many scenarios per GPU (C4 default: strong scaling, see --total-batch)")
    ap.add_argument("--total-batch", type=int, default=None,
                    help="strong scaling: this many scenarios in total, split over the ranks (C4 default when --batch "
                         "is not given: BASELINE configs[3], 65536 across the GPUs, 8192 per GPU at N = 8); the "
                         "same global scenario set for every N")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--mode", default=None)
    ap.add_argument("--forests", type=int, default=64)
    ap.add_argument("--start", choices=["path", "edge"], default="path",
                    help="path: scenarios spread along the forest crossing (default); edge: all at the forest edge")
    ap.add_argument("--config", choices=["C1", "C2", "C3", "C4", "C5"], default="C4",
                    help="SURVEY.md 8(d) workload; C4 (default) is the headline closed loop, C2/C3/C5 are the "
                         "QP-level configs (n, mode, batch and parameters follow the config unless given)")
    ap.add_argument("--fixed-work", action="store_true",
                    help="C2/C5 mode (ii): tol 0, 25 ADMM iterations (test/control/test_rqpcontrollers.py:106-110)")
    ap.add_argument("--fused", action="store_true",
                    help="C2/C3/C5: the timed steps as ONE dat_control_steps call (each scenario starts its next "
                         "control step as soon as its previous one ends; ms_per_step = elapsed / steps)")
    ap.add_argument("--sub-batches", type=int, default=None,
                    help="C4: run each GPU's scenarios as this many sub-batches on their own streams "
                         "(dat_set_sub_batches; per-scenario arithmetic unchanged).  Default: 1 when a GPU holds "
                         ">= 65,536 scenarios, else 4 (auto_sub_batches)")
    ap.add_argument("--qp-tol", type=float, default=1e-10,
                    help="IPM stopping tolerance of the QPs (default 1e-10; 1e-8 = Clarabel's default, which "
                         "the reference runs with)")
    ap.add_argument("--sustained-steps", type=int, default=1000,
                    help="after the timed steps: the closed loop from the start states over this many HL steps "
                         "(SURVEY 8(d)'s 10 s), reported per block of --sustained-block steps (stats.sustained); 0: off")
    ap.add_argument("--sustained-block", type=int, default=100)
    ap.add_argument("--persistent-blocks", type=int, default=0,
                    help="resident k_cadmm / k_dd workgroups (0: the library default, 4 per CU); more workgroups "
                         "hold fewer scenario slots each (dat_set_persistent_blocks)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-s", type=float, default=15.0)
    ap.add_argument("--selftest", action="store_true",
                    help="CPU-only check of the launch / shard / combine path (gloo, no solver work, synthetic numbers)")
    args = ap.parse_args()
    n, mode, batch = QP_CONFIGS.get(args.config, (6, "cadmm", 65536))
    args.n = n if args.n is None else args.n
    args.mode = mode if args.mode is None else args.mode
    if args.config == "C4" and args.batch is None and args.total_batch is None:
        # the headline measures BASELINE configs[3] at every N: 65,536 scenarios split over the ranks
        # (N = 1 runs the same 65,536 scenarios as the weak mode's rank 0)
        args.total_batch = batch
    args.batch = batch if args.batch is None else args.batch
    return args


# (n, controller, scenarios per GPU) of the QP-level configs
QP_CONFIGS = {"C2": (3, "cadmm", 1024), "C3": (6, "dd", 16384), "C5": (16, "cadmm", 32768),
              # config 1's controller (example/rqp_example.py: centralized, n = 3) batched over scenarios
              "C1": (3, "centralized", 65536)}
ACC_POOL = 8  # distinct acc_des draws cycled over the timed steps


def qp_level_inputs(cfg: str, n: int, batch: int, rng: np.random.Generator):
    """C2/C3/C5 inputs: perturbed rest states (scenarios.perturbed_states), acc_des ~ U(-5, 5)^6
    (test/control/test_rqpcontrollers.py:117-118); C3 adds per-scenario payload mass / inertia."""
    from distributed_aerial_transportation_amd import scenarios

    states = scenarios.perturbed_states(n, batch, rng)
    accs = [rng.uniform(-0.5, 0.5, (batch, 6)) * 10.0 for _ in range(ACC_POOL)]
    if cfg == "C3":
        return states, accs, scenarios.randomized_params(n, batch, rng), True
    return states, accs, scenarios.params_block(n), False


def cpu_baseline_qp(cfg: str, n: int, mode: str, budget_s: float, fixed_work: bool):
    """Oracle (numpy) controller on a bounded sample of the same QP-level workload, one core."""
    from distributed_aerial_transportation_amd import scenarios
    from distributed_aerial_transportation_amd.system import RQPState
    from oracle import controllers as oc
    from oracle import model as om
    from oracle import scenarios as osc

    rng = np.random.default_rng(321)
    solves, steps, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        x = scenarios.perturbed_states(n, 1, rng)[0]
        acc = rng.uniform(-0.5, 0.5, 6) * 10.0
        m, J, ml, Jl, r = osc.geometry(n)
        if cfg == "C3":
            ml, Jl = rng.uniform(0.15, 0.30), Jl * np.diag(rng.uniform(0.8, 1.2, 3))
        p = om.Params(m, J, ml, Jl, r)
        ctl = {"dd": oc.DD, "cadmm": oc.CADMM, "centralized": oc.Centralized}[mode](p, osc.col_radius(n))
        if fixed_work and mode == "cadmm":
            ctl.set_force_err_tolerance(0.0, False)
            ctl.set_max_iter(25)
        s = RQPState.unpack(x, n)
        _, st = ctl.control(om.State(s.R, s.w, s.xl, s.vl, s.Rl, s.wl, project=False), (acc[:3], acc[3:]))
        solves += 1 if mode == "centralized" else st.iter * n
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": solves / dt, "unit": "agent-QP solves/s", "cores": 1, "kind": "port",
            "sample": f"oracle {mode} n={n} (numpy dense IPM), {steps} cold control steps of {cfg} inputs, "
                      f"{solves} {'centralized' if mode == 'centralized' else 'agent'} QPs in {dt:.1f} s"}


def cpu_baseline(n: int, budget_s: float, start: str, forests_n: int, warmup: int, steps: int, batch: int,
                 late_steps: int = 0, late_block: int = 100):
    """The C4 closed loop on this host's cores (cpu_baseline/: the same per-scenario C-ADMM loop and
    per-lane fp64 code as the GPU, OpenMP over scenarios, -O3 x86-64-v3), work-matched to the GPU
    line: the first S of rank 0's scenarios -- the same start states, forests and controller -- run
    the bench's `warmup` untimed HL steps and then exactly its `steps` timed HL steps (desired
    acceleration + C-ADMM control + 10 simulation steps), so the CPU solves the same agent QPs from the
    same warm states as the GPU's timed region (S = all of them unless that exceeds ~budget_s; a
    1-step calibration on a small subset sizes S).  Once on all OpenMP threads of this process (the
    reported value) and once on 1 thread (the first 64 scenarios).  late_steps > 0: the late loop as well
    (late_loop): the first S2 scenarios run HL steps [0, late_steps - late_block) untimed and the last block
    timed, the window of the GPU's last sustained block (S2 sized to ~1/4 of budget_s at the warm rate)."""
    import cpu_baseline as cb
    from distributed_aerial_transportation_amd import Forest, scenarios

    cb.build()
    threads = cb.CpuClosedLoop.max_threads()
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count()
    scen_forest, states, forests = bench_states(n, batch, 0, 1, forests_n, start, None)
    params = scenarios.params_block(n)

    def ctx(count):
        c = cb.CpuClosedLoop(n, count, params)
        c.set_forests(forests, scen_forest[:count])
        c.set_state(states[:count])
        return c

    # calibration: one HL step of a small subset from the start states (scenario-steps per second)
    S0 = min(batch, 32 * threads)
    cal = ctx(S0)
    t0 = time.perf_counter()
    cal.closed_loop(1, threads=threads)
    rate = S0 / max(time.perf_counter() - t0, 1e-6)
    cal.close()
    S = int(min(batch, max(S0, budget_s * rate / max(steps, 1))))
    c = ctx(S)
    c.closed_loop(warmup, threads=threads)  # the GPU line's untimed warm-up steps
    t0 = time.perf_counter()
    qN, iN = c.closed_loop(steps, threads=threads)
    tN = time.perf_counter() - t0
    c.close()
    S1 = min(S, 64)
    c1 = ctx(S1)
    c1.closed_loop(warmup, threads=1)
    t0 = time.perf_counter()
    q1, _ = c1.closed_loop(steps, threads=1)
    t1 = time.perf_counter() - t0
    c1.close()
    late = None
    if late_steps > late_block > 0:
        rate_warm = S * steps / max(tN, 1e-6)  # scenario-steps per second of the timed (warm) steps
        S2 = int(min(batch, max(threads, 0.25 * budget_s * rate_warm / late_steps)))
        c2 = ctx(S2)
        c2.closed_loop(late_steps - late_block, threads=threads)
        t0 = time.perf_counter()
        q2, i2 = c2.closed_loop(late_block, threads=threads)
        t2 = time.perf_counter() - t0
        c2.close()
        late = {"value": q2 / t2, "unit": "agent-QP solves/s", "cores": threads,
                "ms_per_scenario_step": t2 * 1e3 / (S2 * late_block) * threads,
                "sample": f"the first {S2} scenarios, HL steps {late_steps - late_block}-{late_steps - 1} of the "
                          f"closed loop from the start states ({q2} agent QPs, {i2 / max(q2, 1):.2f} IPM it/QP, "
                          f"{t2:.1f} s on {threads} threads)"}
    try:
        cpu = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except (OSError, IndexError):
        cpu = "unknown"
    return {"value": qN / tN, "unit": "agent-QP solves/s", "cores": threads, "affinity_cpus": affinity,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "kind": "port", "single_core_value": q1 / t1, "ipm_iters_per_qp": iN / max(qN, 1), "late_loop": late,
            "sample": f"C++ OpenMP restatement of the C4 loop (cpu_baseline/dat_cpu.hip, same per-lane code as the "
                      f"kernels), n={n}: the first {S} of the bench's {batch} {start}-start scenarios (rank 0), "
                      f"{warmup} untimed + {steps} timed HL steps like the GPU line ({qN} agent QPs, "
                      f"{iN / max(qN, 1):.2f} IPM it/QP, {tN:.1f} s) on {threads} OpenMP threads "
                      f"(omp_get_max_threads, OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}: the "
                      f"box's CPU share; sched_getaffinity: {affinity} CPUs); 1 thread: {S1} scenarios x {steps} steps "
                      f"({q1} QPs); host CPU {cpu}, os.cpu_count() {os.cpu_count()}"}


def shard(rank: int, batch: int, num_forests: int):
    """Scenario range of one rank (weak scaling): global scenario ids [rank B, (rank + 1) B); scenario
    s drives forest s mod num_forests; start states from a per-rank seed."""
    ids = np.arange(batch) + rank * batch
    return ids % num_forests, 1000 + rank


def strong_shard(rank: int, world: int, total: int):
    """Strong scaling: contiguous split of `total` scenario ids over `world` ranks (the first
    total % world ranks take one more): the package's sharding.shard_range."""
    from distributed_aerial_transportation_amd.sharding import shard_range

    return shard_range(rank, world, total)


def bench_states(n: int, batch: int, rank: int, world: int, forests_n: int, start: str, total):
    """(scenario_forest, start states, forests) of one rank.  Weak scaling (total None): `batch`
    scenarios from the per-rank seed (shard).  Strong scaling: the global set of `total` scenarios from
    one seed, every rank taking its contiguous slice (strong_shard), so every N runs the same scenarios."""
    from distributed_aerial_transportation_amd import Forest, scenarios

    forests = [Forest.seeded(s) for s in range(forests_n)]
    if total is None:
        sf, seed = shard(rank, batch, forests_n)
        ids, count = None, batch
    else:
        lo, cnt = strong_shard(rank, world, total)
        sf, seed = shard(0, total, forests_n)
        ids, count = slice(lo, lo + cnt), total
    rng = np.random.default_rng(seed)
    if start == "path":
        st = scenarios.forest_path_states(n, count, rng, forests, sf)
    else:
        st = scenarios.forest_start_states(n, count, rng)
    if ids is not None:
        sf, st = sf[ids], st[ids]
    return np.ascontiguousarray(sf), np.ascontiguousarray(st), forests


def combine_ranks(comm, tot: np.ndarray, metrics: np.ndarray):
    """Sum of the work counters, max of the elapsed time, all-gather of the per-scenario metrics (uneven
    shards included) through the package's sharding collectives.  The only collectives of the run (RCCL
    over xGMI: sharding.Comm; the gloo test harness on CPU)."""
    from distributed_aerial_transportation_amd.sharding import gather_rows, reduce_values

    return reduce_values(tot, "sum", comm), reduce_values(tot, "max", comm), gather_rows(metrics, comm)


def spawn_ranks(args) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes (one per GPU) with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, exactly as torch.distributed.run would, and exit
    with the worst rank's code.  This parent process never touches the GPU (no HIP call, no
    torch.cuda), so the ranks own their devices; rank 0 prints the JSON line."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


class _SelftestEngine:
    """--selftest: stands in for BatchedController so the launch / sharding / rank-combination path of
    this script can be exercised on a CPU-only host (gloo).  It performs no solver work and its
    numbers are synthetic; the JSON line says so ("data": "selftest")."""

    def __init__(self, n: int, batch: int, rank: int) -> None:
        self.n, self.batch, self.rank, self.steps = n, batch, rank, 0

    def set_forests(self, *a, **k):
        pass

    def set_state(self, *a, **k):
        pass

    def closed_loop(self, k):
        self.steps += k

    def step_marks(self):
        return np.arange(self.steps + 1, dtype=np.float64)

    def reset_counters(self):
        self.steps = 0

    def synchronize(self):
        pass

    def work(self):
        q = self.steps * self.batch * self.n
        return {"qp_solves": q, "ipm_iters": 7 * q, "ipm_row_iters": 35 * q, "hl_steps": self.steps,
                "hl_kernel_ms": 1.0 * self.steps}

    def class_work(self, k):
        w = self.work()
        return dict(w, kernel_ms=w["hl_kernel_ms"], slot_ipm_iters=w["ipm_iters"], wave_admm_iters=w["qp_solves"] // self.n)

    def control(self, *a):
        from types import SimpleNamespace

        return SimpleNamespace(iters=np.full(self.batch, 1 + self.rank, dtype=np.int32),
                               min_env_dist=np.full(self.batch, 1.0), collision=np.zeros(self.batch, dtype=bool),
                               qp_status=np.zeros((self.batch, self.n), dtype=np.int32))


def timed_steps(eng, steps: int, barrier):
    """Run `steps` closed-loop HL periods back to back in one dat_closed_loop call, bracketed by the
    barrier + device synchronisation; returns (elapsed s, per-step ms array).  The per-step times are
    the library's host clock marks at each step's control-kernel completion (dat_get_step_marks): the
    host enqueues step k + 1 while step k's rollout runs, so no per-step host round trip is timed."""
    barrier()
    eng.synchronize()
    t0 = time.perf_counter()
    eng.closed_loop(steps)
    eng.synchronize()
    t1 = time.perf_counter()
    barrier()
    marks = eng.step_marks()
    per = np.diff(marks) if len(marks) == steps + 1 else np.full(steps, (t1 - t0) * 1e3 / steps)
    return t1 - t0, per


def sustained_loop(eng, states, steps: int, block: int, barrier, comm, n: int, batch_all: int) -> dict:
    """SURVEY 8(d)'s sustained rate: the closed loop from the start states (warm state reset) over `steps` HL
    steps, timed per block of `block` steps like the timed region (barrier + device synchronisation around
    one dat_closed_loop call; max over ranks, counters summed).  The late blocks hold the stalled ADMM loops
    next to trees that the short timed region does not reach (their agent QPs take the robust redo)."""
    eng.reset_warm_start()
    eng.set_state(states, np.zeros(len(states), dtype=np.int32))
    rows = []
    for b0 in range(0, steps, block):
        k = min(block, steps - b0)
        eng.reset_counters()
        barrier()
        eng.synchronize()
        t0 = time.perf_counter()
        eng.closed_loop(k)
        eng.synchronize()
        dt = time.perf_counter() - t0
        barrier()
        w = eng.work()
        # (the minimum env distance enters as its negative, so that one "max" reduction carries both maxima)
        rows.append([dt, w["qp_solves"], w["ipm_iters"], w.get("inband_exits", 0),
                     w.get("inband_beyond_clarabel_tol", 0), w.get("robust_redos", 0), k, w.get("collisions", 0),
                     -w.get("min_env_dist", np.inf), w.get("tail_routed", 0), w.get("certified_infeasible", 0),
                     w.get("stall_exits", 0), w.get("tail_passes", 0), w.get("tail_critical_ipm_iters", 0)])
    rows = np.array(rows, dtype=np.float64)
    if comm is not None:
        from distributed_aerial_transportation_amd.sharding import reduce_values

        mx = reduce_values(rows.reshape(-1), "max", comm).reshape(rows.shape)
        rows = reduce_values(rows.reshape(-1), "sum", comm).reshape(rows.shape)
        rows[:, 0], rows[:, 6], rows[:, 8] = mx[:, 0], mx[:, 6], mx[:, 8]
    blocks = []
    b0 = 0
    for dt, q, ip, ib, lo, rr, k, col, nmd, trt, cert, stx, tps, tcr in rows:
        blocks.append({"hl_steps": f"{b0}-{b0 + int(k) - 1}", "ms_per_step": dt / k * 1e3, "qp_per_s": q / dt,
                       "mean_admm_passes": q / (batch_all * n * k), "ipm_iters_per_qp": ip / max(q, 1),
                       "inband_exits": int(ib), "inband_beyond_clarabel_tol": int(lo), "robust_redos": int(rr),
                       # scenario-steps with the reference's collision flag (example/env_forest.py:158-159) and the
                       # smallest min env distance of the block (example/rqp_example.py:129)
                       "collisions": int(col), "min_env_dist": float(-nmd),
                       # the tail (k_cadmm_tail): scenario-steps routed before the step, agent QPs certified
                       # infeasible, stall exits, its passes and their critical-path IPM iterations
                       "tail_routed": int(trt), "certified_infeasible": int(cert), "stall_exits": int(stx),
                       "tail_passes": int(tps), "tail_critical_ipm_per_pass": tcr / max(tps, 1)})
        b0 += int(k)
    T, Q = rows[:, 0].sum(), rows[:, 1].sum()
    return {"hl_steps": steps, "block": block, "ms_per_step": T / steps * 1e3, "qp_per_s": Q / T,
            "slowest_block_ms_per_step": max(b["ms_per_step"] for b in blocks),
            "inband_beyond_clarabel_tol": int(rows[:, 4].sum()), "robust_redos": int(rows[:, 5].sum()),
            "collisions": int(rows[:, 7].sum()), "min_env_dist": float(-rows[:, 8].max()),
            "blocks": blocks}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    comm = None
    if world > 1:
        if args.selftest:  # CPU-only check of the launch / shard / combine path: the gloo test harness
            import torch.distributed as tdist

            from tests._gloo_comm import GlooComm

            tdist.init_process_group("gloo", init_method="env://")
            comm = GlooComm()
        else:  # RCCL over xGMI through libdat.so (no PyTorch in the rank processes)
            from distributed_aerial_transportation_amd.sharding import Comm

            comm = Comm.from_env(device=local)

    if args.config != "C4":
        if args.selftest:
            sys.exit("bench.py: --selftest covers the C4 path only")
        return qp_level(args, comm, rank, world, local)
    n = args.n
    total = args.total_batch
    B = args.batch if total is None else strong_shard(rank, world, total)[1]
    if args.sub_batches is None:
        args.sub_batches = min(auto_sub_batches(B), max(B, 1))
    if args.selftest:
        eng = _SelftestEngine(n, B, rank)
    else:
        from distributed_aerial_transportation_amd import BatchedController, scenarios

        scen_forest, states, forests = bench_states(n, B, rank, world, args.forests, args.start, total)
        eng = BatchedController(args.mode, n, B, scenarios.params_block(n), device=local if world > 1 else 0)
        eng.set_qp_tolerance(args.qp_tol)
        if args.persistent_blocks:
            eng.set_persistent_blocks(args.persistent_blocks)
        eng.set_forests(forests, scen_forest)
        eng.set_state(states, np.zeros(B, dtype=np.int32))
        if args.sub_batches > 1:
            eng.set_sub_batches(args.sub_batches)
    eng.closed_loop(args.warmup)
    eng.reset_counters()

    def barrier():
        if comm is not None:
            comm.barrier()  # (RCCL: every stream of the rank drained first)

    elapsed, per_step = timed_steps(eng, args.steps, barrier)
    elapsed_rank0 = elapsed
    work = eng.work()
    qps, ipm, hl_steps, hl_ms = work["qp_solves"], work["ipm_iters"], work["hl_steps"], work["hl_kernel_ms"]
    row_it = work["ipm_row_iters"]
    # per-class counters and the k_cadmm event time of the timed steps, read before the metrics step
    # below (its launch is not part of the timed region)
    class_w = [eng.class_work(k) for k in range(4)] if args.mode == "cadmm" else None
    # per-scenario metrics of the last step (all-gathered over ranks: the only collective)
    res = eng.control(None, None)
    # per scenario: outer iterations, min env distance, collision flag, agent QPs not OPTIMAL
    local_metrics = np.stack([res.iters.astype(np.float64), res.min_env_dist, res.collision.astype(np.float64),
                              (np.asarray(res.qp_status) != 0).sum(axis=1).astype(np.float64)], 1)
    tot = np.array([qps, ipm, hl_ms, elapsed, row_it, work.get("inband_exits", 0), B,
                    work.get("inband_beyond_clarabel_tol", 0)], dtype=np.float64)
    if comm is not None:
        sums, maxs, all_metrics = combine_ranks(comm, tot, local_metrics)
        qps_all, ipm_all, row_all = float(sums[0]), float(sums[1]), float(sums[4])
        inband_all, scen_all, loose_all = int(sums[5]), int(sums[6]), int(sums[7])
        elapsed = float(maxs[3])
        hl_ms_rank0 = float(tot[2])
    else:
        all_metrics = local_metrics
        qps_all, ipm_all, row_all, hl_ms_rank0 = float(qps), float(ipm), float(row_it), float(hl_ms)
        inband_all, scen_all, loose_all = int(tot[5]), B, int(tot[7])
    sust = None
    if args.sustained_steps > 0 and not args.selftest:
        sust = sustained_loop(eng, states, args.sustained_steps, args.sustained_block, barrier, comm, n, scen_all)
    if rank != 0:
        if comm is not None:
            comm.close()
        return
    value = qps_all / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    launch_ms = hl_ms_rank0 / max(hl_steps, 1)
    # roofline of the dominant kernel, rank 0's own launches: algorithmic flops of one launch / its
    # average duration (HIP events on the handle's stream).  C-ADMM: k_cadmm (env classes 0..3: no
    # env rows, up to 2 / 5 / 10 env rows per agent QP, all drained by one persistent launch).
    kernel, k_ipm, k_row, k_ms, classes = "k_cadmm", ipm, row_it, hl_ms, None
    if args.mode == "cadmm":
        # one persistent k_cadmm launch per control step drains the four env classes
        classes = {}
        for k in range(4):
            w = class_w[k]
            classes[f"class{k}"] = {"qp_solves": w["qp_solves"], "ipm_iters": w["ipm_iters"],
                                    "mean_active_rows": w["ipm_row_iters"] / max(w["ipm_iters"], 1),
                                    # useful lane-iterations / lane-iterations the wavefronts ran
                                    "ipm_lane_utilisation": w["ipm_iters"] / max(w["slot_ipm_iters"], 1),
                                    "admm_slot_utilisation": w["qp_solves"] / n / max(w["wave_admm_iters"], 1)}
            k_ms = w["kernel_ms"]
    # k_cadmm launches per HL step: one per sub-batch stream
    launches = max(hl_steps, 1) * max(args.sub_batches, 1)
    kernel_ms = k_ms / launches
    # (with sub-batch streams: one k_cadmm launch per sub-batch and step, each timed by its own event pair on
    # its stream; the roofline is per launch, launches_per_step says how many)
    flops_launch = model_flops(args.mode, n, k_ipm, k_row, work.get("refine_passes", 0),
                               work.get("refine_corrections", 0)) / launches
    achieved_tflops = flops_launch / max(kernel_ms * 1e-3, 1e-12) / 1e12
    per_launch_tflops = None
    if args.sub_batches > 1:
        # concurrent sub-batch launches share the device: each launch's event span also covers the others'
        # work, so the per-launch figure understates the device's rate.  The roofline is then device-level:
        # the flops of every launch of the timed steps over the timed region (rank 0)
        per_launch_tflops = achieved_tflops
        achieved_tflops = flops_launch * launches / max(elapsed_rank0, 1e-12) / 1e12
    if total is None:
        workload = f"C4: {args.mode} n={n}, forest env ({args.start} start), {B} closed-loop scenarios per GPU"
    else:
        workload = (f"C4: {args.mode} n={n}, forest env ({args.start} start), {total} closed-loop scenarios split "
                    f"over {world} GPU(s)")
    if args.sub_batches > 1:
        workload += f", {args.sub_batches} sub-batch streams per GPU"

    traffic, traffic_src = traffic_per_launch(kernel, workload)
    out = {
        "metric": "agent-QP solves/sec (node) + ms per control step, 6-quad C-ADMM, 1/2/4/8 GPU",
        "value": value,
        "unit": "agent-QP solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        # (sub-batch streams run their steps independently: no per-step marks, no percentiles)
        "ms_per_step_p50": None if args.sub_batches > 1 else float(np.percentile(per_step, 50)),
        "ms_per_step_p99": None if args.sub_batches > 1 else float(np.percentile(per_step, 99)),
        "higher_is_better": True,
        "scaling": "weak" if total is None else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("selftest (no solver work; synthetic counters)" if args.selftest else
                 f"synthetic (seeded forests 0..63, randomized C4 {args.start} start states)"),
        "config": {"workload": workload,
                   "n": n, "scenarios_per_gpu": B, "total_scenarios": scen_all, "hl_every": 10, "dt": 1e-3,
                   "qp_tol": args.qp_tol, "parallelism": f"scenario-sharded x{world}",
                   "sub_batches": args.sub_batches, "persistent_blocks": args.persistent_blocks or "default"},
        "stats": {"agent_qp_solves": qps_all, "ipm_iters": ipm_all, "mean_ipm_iters_per_qp": ipm_all / max(qps_all, 1),
                  "mean_active_rows": row_all / max(ipm_all, 1),
                  "mean_admm_iters": float(np.mean(all_metrics[:, 0])), "collisions_last_step": int(all_metrics[:, 2].sum()),
                  "non_optimal_agent_qps_last_step": int(all_metrics[:, 3].sum()),
                  "hl_kernel_ms_per_step": launch_ms, "env_classes": classes,
                  # agent QPs accepted through the best in-band iterate, and those beyond Clarabel's
                  # 1e-8 tolerance (dat_get_inband_exits)
                  "inband_exits": inband_all, "inband_beyond_clarabel_tol": loose_all,
                  # scenario-steps k_cadmm handed to k_cadmm_rob (an agent QP not clean), rank 0
                  "robust_redos": int(work.get("robust_redos", 0)),
                  # the 10 s closed loop from the start states, per block of HL steps (sustained_loop)
                  "sustained": sust},
        "roofline": {"bound": "fp64-valu", "achieved": achieved_tflops, "peak": FP64_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved_tflops / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "traffic_source": traffic_src, "kernel": kernel, "launch_ms": kernel_ms,
                     "scope": "device (all sub-batch launches / timed region)" if args.sub_batches > 1 else "per launch",
                     "per_launch_achieved": per_launch_tflops,
                     "launches_per_step": max(args.sub_batches, 1),
                     "flops_per_launch": flops_launch, "flop_model": model_string(args.mode)},
    }
    # (the CPU restatement solves at the default 1e-10: no work-matched baseline at another --qp-tol)
    if not args.no_cpu_baseline and world == 1 and not args.selftest and args.qp_tol == 1e-10:
        out["cpu_baseline"] = cpu_baseline(n, args.cpu_sample_s, args.start, args.forests, args.warmup, args.steps, B,
                                           args.sustained_steps, args.sustained_block)
    print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()


def qp_level(args, comm, rank: int, world: int, local: int):
    """C2 / C3 / C5: one step = one batched control step of every scenario from HBM-resident states
    (no rollout, no env).  acc_des cycles through ACC_POOL pre-drawn arrays; its host-to-device copy
    (48 B per scenario) is inside the timed region.  Warm state (f, f_bar, lambda / lambda_F,M)
    persists across steps as in the reference controller objects."""
    from distributed_aerial_transportation_amd import BatchedController, _lib as L

    n, B, cfg = args.n, args.batch, args.config
    rng = np.random.default_rng(2000 + rank)
    states, accs, params, per_scen = qp_level_inputs(cfg, n, B, rng)
    eng = BatchedController(args.mode, n, B, params, per_scenario_params=per_scen,
                            device=local if world > 1 else 0)
    eng.set_qp_tolerance(args.qp_tol)
    if args.persistent_blocks:
        eng.set_persistent_blocks(args.persistent_blocks)
    if args.fixed_work:
        eng.set_force_err_tolerance(0.0, False)
        eng.set_max_iter(25)
    eng.set_state(states)
    accs = [L.f64(a) for a in accs]
    lib, h = eng._lib, eng._h

    def step(k):
        L.check(lib.dat_control_step(h, None, L.ptr(accs[k % ACC_POOL]), None, None, None, None, None, None))

    def fused(k0, K):
        seq = L.f64(np.stack([accs[(k0 + k) % ACC_POOL] for k in range(K)]))
        L.check(lib.dat_control_steps(h, K, L.ptr(seq), None, None, None))

    if args.fused and args.mode == "centralized":
        sys.exit("bench.py: --fused covers the C-ADMM / DD configs")
    if args.fused:
        if args.warmup:
            fused(0, args.warmup)
    else:
        for k in range(args.warmup):
            step(k)
    eng.synchronize()
    eng.reset_counters()

    def barrier():
        if comm is not None:
            comm.barrier()

    barrier()
    eng.synchronize()
    per_step = np.full(args.steps, np.nan)
    t0 = time.perf_counter()
    if args.fused:  # (the K x B x 6 host-to-device copy of the acc sequence is inside the timed region)
        fused(args.warmup, args.steps)
        eng.synchronize()
    else:
        for k in range(args.steps):
            ts = time.perf_counter()
            step(args.warmup + k)
            eng.synchronize()
            per_step[k] = (time.perf_counter() - ts) * 1e3
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    w = eng.work()
    kms = eng.kernel_ms()  # k_cadmm / k_dd of the timed steps (before the metrics-only step below)
    res = eng.control(None, L.f64(accs[0]))  # metrics only (outside the timed region)
    # per scenario: outer iterations, min env distance, collision flag, agent QPs not OPTIMAL
    local_metrics = np.stack([res.iters.astype(np.float64), res.min_env_dist, res.collision.astype(np.float64),
                              (np.asarray(res.qp_status) != 0).sum(axis=1).astype(np.float64)], 1)
    tot = np.array([w["qp_solves"], w["ipm_iters"], w["hl_kernel_ms"], elapsed, w["ipm_row_iters"]])
    if comm is not None:
        sums, maxs, all_metrics = combine_ranks(comm, tot, local_metrics)
        qps, ipm, rows, elapsed = float(sums[0]), float(sums[1]), float(sums[4]), float(maxs[3])
    else:
        all_metrics = local_metrics
        qps, ipm, rows = float(tot[0]), float(tot[1]), float(tot[4])
    if rank != 0:
        if comm is not None:
            comm.close()
        return
    # (the QP-level configs have no forest: the C-ADMM drain is the class-0 kernel k_cadmm0)
    kernel = {"cadmm": "k_cadmm0", "dd": "k_dd", "centralized": "k_cent"}.get(args.mode, args.mode)
    step_ms = float(tot[2]) / max(w["hl_steps"], 1)
    launch_ms = kms / max(w["hl_steps"], 1) if args.mode != "centralized" else step_ms
    flops_launch = model_flops(args.mode, n, float(tot[1]), float(tot[4]), w.get("refine_passes", 0),
                               w.get("refine_corrections", 0)) / max(w["hl_steps"], 1)
    tflops = flops_launch / max(launch_ms * 1e-3, 1e-12) / 1e12
    work_mode = "fixed work: tol 0, 25 ADMM iterations" if args.fixed_work else "reference loop: tol 1e-2, max_iter 100"
    if args.mode == "centralized":
        work_mode = "one centralized QP per scenario and step"
    workload = f"{cfg}: {args.mode} n={n}, QP-level, no env ({work_mode}), {B} scenarios per GPU"
    if args.fused:
        workload += f", {args.steps} control steps fused into one drain (dat_control_steps)"
    out = {
        "metric": "agent-QP solves/sec (node) + ms per control step, 6-quad C-ADMM, 1/2/4/8 GPU",
        "value": qps / elapsed, "unit": "centralized-QP solves/s" if args.mode == "centralized" else "agent-QP solves/s",
        "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "ms_per_step_p50": None if args.fused else float(np.percentile(per_step, 50)),
        "ms_per_step_p99": None if args.fused else float(np.percentile(per_step, 99)),
        "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (perturbed rest states, acc_des ~ U(-5,5)^6" + (", randomized payload mass/inertia)" if per_scen else ")"),
        "config": {"workload": workload, "n": n, "scenarios_per_gpu": B, "qp_tol": args.qp_tol,
                   "parallelism": f"scenario-sharded x{world}", "persistent_blocks": args.persistent_blocks or "default"},
        "stats": {"agent_qp_solves": qps, "ipm_iters": ipm, "mean_ipm_iters_per_qp": ipm / max(qps, 1),
                  "mean_active_rows": rows / max(ipm, 1), "mean_admm_iters": float(np.mean(all_metrics[:, 0])),
                  "non_optimal_agent_qps_last_step": int(all_metrics[:, 3].sum()),
                  "kernel_ms_per_step": step_ms, "inband_exits": int(w.get("inband_exits", 0)),
                  "inband_beyond_clarabel_tol": int(w.get("inband_beyond_clarabel_tol", 0))},
        "roofline": {"bound": "fp64-valu", "achieved": tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": tflops / FP64_PEAK_TFLOPS, "traffic": None, "kernel": kernel, "launch_ms": launch_ms,
                     "flops_per_launch": flops_launch,
                     "flop_model": model_string(args.mode) + (" (DD agent QP; dual ascent not counted)"
                                                              if args.mode == "dd" else "")},
    }
    if not args.no_cpu_baseline and world == 1 and args.qp_tol == 1e-10:
        out["cpu_baseline"] = cpu_baseline_qp(cfg, n, args.mode, args.cpu_sample_s, args.fixed_work)
    print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()


if __name__ == "__main__":
    main()
