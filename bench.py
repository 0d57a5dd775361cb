"""Benchmark: agent-QP solves/s (node) + ms per control step, 6-quadrotor C-ADMM (BASELINE.json).

Workload (per GPU): n = 6 C-ADMM in the forest environment, B = 65536
closed-loop scenarios per GPU (weak scaling), 64 seeded forests (scenario s uses forest s mod 64),
start xl = (U(-2,0), U(-10,10), 1.5), vl = (0.5, 0, 0).  One "step" = one high-level period of
every scenario, fully on device: forest desired-acceleration law + C-ADMM control step (env CBF
rows, up to 101 ADMM iterations of n agent QPs each) + 10 simulation steps (SO(3) PD + dynamics).

    python bench.py [--gpus N --steps K --warmup W --batch B --n 6 --mode cadmm]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

The data path has no collective; torch.distributed (RCCL over xGMI when N > 1) is used for the
barrier, the max-over-ranks time and an all-gather of the per-scenario metrics.
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
# Algorithmic FP64 flops per IPM iteration of the reduced C-ADMM agent QP:
# F_it(R) = FLOPS_FIXED + FLOPS_PER_ROW * R, R = active constraint rows of the solve.  The kernel
# counts IPM iterations and IPM iterations x active rows on device (dat_get_counters).
FLOPS_FIXED = 7267.0
FLOPS_PER_ROW = 283.0
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=65536, help="scenarios per GPU")
    ap.add_argument("--n", type=int, default=6)
    ap.add_argument("--mode", default="cadmm")
    ap.add_argument("--forests", type=int, default=64)
    ap.add_argument("--start", choices=["path", "edge"], default="path",
                    help="path: scenarios spread along the forest crossing (default); edge: all at the forest edge")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-s", type=float, default=15.0)
    return ap.parse_args()


def cpu_baseline(n: int, budget_s: float, start: str = "path"):
    """Oracle (numpy) C-ADMM on a bounded sample of the same workload, one core."""
    from distributed_aerial_transportation_amd import Forest, scenarios
    from distributed_aerial_transportation_amd.system import RQPState
    from oracle import controllers as oc
    from oracle import forest as of
    from oracle import model as om
    from oracle import scenarios as osc

    rng = np.random.default_rng(123)
    np.random.seed(0)
    forest = of.Forest()
    layout = Forest.seeded(0)  # the same seed-0 tree layout, with the terrain helper for the start heights
    solves, t0, steps = 0, time.perf_counter(), 0
    while time.perf_counter() - t0 < budget_s:
        if start == "path":
            x = scenarios.forest_path_states(n, 1, rng, [layout], np.zeros(1, dtype=int))[0]
        else:
            x = scenarios.forest_start_states(n, 1, rng)[0]
        s = RQPState.unpack(x, n)
        st = om.State(s.R, s.w, s.xl, s.vl, s.Rl, s.wl, project=False)
        ctl = oc.CADMM(osc.params(n), osc.col_radius(n), forest)
        acc, _, _ = oc.desired_acceleration_forest(st, forest)
        _, stats = ctl.control(st, acc)
        solves += stats.iter * n
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": solves / dt, "unit": "agent-QP solves/s", "cores": 1, "kind": "port",
            "sample": f"oracle C-ADMM n={n} (numpy dense IPM), {steps} forest control steps from C4 start "
                      f"states ({start} start), {solves} agent QPs in {dt:.1f} s"}


def shard(rank: int, batch: int, num_forests: int):
    """Scenario range of one rank (weak scaling): global scenario ids [rank B, (rank + 1) B); scenario
    s drives forest s mod num_forests; start states from a per-rank seed."""
    ids = np.arange(batch) + rank * batch
    return ids % num_forests, 1000 + rank


def combine_ranks(dist, world: int, tot: np.ndarray, metrics: np.ndarray, device):
    """Sum of the work counters, max of the elapsed time, all-gather of the per-scenario metrics.
    The only collectives of the run (RCCL over xGMI with the nccl backend; gloo on CPU in tests)."""
    import torch

    t = torch.tensor(tot, dtype=torch.float64, device=device)
    mx = t.clone()
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    gm = torch.tensor(metrics, dtype=torch.float64, device=device)
    gath = [torch.empty_like(gm) for _ in range(world)]
    dist.all_gather(gath, gm)
    return t.cpu().numpy(), mx.cpu().numpy(), torch.cat(gath).cpu().numpy()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    from distributed_aerial_transportation_amd import BatchedController, Forest, scenarios

    n, B = args.n, args.batch
    scen_forest, seed = shard(rank, B, args.forests)
    rng = np.random.default_rng(seed)
    forests = [Forest.seeded(s) for s in range(args.forests)]
    if args.start == "path":
        states = scenarios.forest_path_states(n, B, rng, forests, scen_forest)
    else:
        states = scenarios.forest_start_states(n, B, rng)
    eng = BatchedController(args.mode, n, B, scenarios.params_block(n), device=local if world > 1 else 0)
    eng.set_forests(forests, scen_forest)
    eng.set_state(states, np.zeros(B, dtype=np.int32))
    eng.closed_loop(args.warmup)
    eng.reset_counters()

    def barrier():
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    barrier()
    eng.synchronize()
    t0 = time.perf_counter()
    eng.closed_loop(args.steps)
    eng.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    work = eng.work()
    qps, ipm, hl_steps, hl_ms = work["qp_solves"], work["ipm_iters"], work["hl_steps"], work["hl_kernel_ms"]
    row_it = work["ipm_row_iters"]
    # per-scenario metrics of the last step (all-gathered over ranks: the only collective)
    res = eng.control(None, None)
    local_metrics = np.stack([res.iters.astype(np.float64), res.min_env_dist, res.collision.astype(np.float64)], 1)
    tot = np.array([qps, ipm, hl_ms, elapsed, row_it], dtype=np.float64)
    if dist is not None:
        sums, maxs, all_metrics = combine_ranks(dist, world, tot, local_metrics, f"cuda:{local}")
        qps_all, ipm_all, row_all = float(sums[0]), float(sums[1]), float(sums[4])
        elapsed = float(maxs[3])
        hl_ms_rank0 = float(tot[2])
    else:
        all_metrics = local_metrics
        qps_all, ipm_all, row_all, hl_ms_rank0 = float(qps), float(ipm), float(row_it), float(hl_ms)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
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
            w = eng.class_work(k)
            classes[f"class{k}"] = {"qp_solves": w["qp_solves"], "ipm_iters": w["ipm_iters"],
                                    "mean_active_rows": w["ipm_row_iters"] / max(w["ipm_iters"], 1),
                                    # useful lane-iterations / lane-iterations the wavefronts ran
                                    "ipm_lane_utilisation": w["ipm_iters"] / max(w["slot_ipm_iters"], 1),
                                    "admm_slot_utilisation": w["qp_solves"] / n / max(w["wave_admm_iters"], 1)}
            k_ms = w["kernel_ms"]
    kernel_ms = k_ms / max(hl_steps, 1)
    flops_launch = (FLOPS_FIXED * k_ipm + FLOPS_PER_ROW * k_row) / max(hl_steps, 1)
    achieved_tflops = flops_launch / max(kernel_ms * 1e-3, 1e-12) / 1e12
    workload = f"C4: {args.mode} n={n}, forest env ({args.start} start), {B} closed-loop scenarios per GPU"
    traffic, traffic_src = traffic_per_launch(kernel, workload)
    out = {
        "metric": "agent-QP solves/sec (node) + ms per control step, 6-quad C-ADMM, 1/2/4/8 GPU",
        "value": value,
        "unit": "agent-QP solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic (seeded forests 0..63, randomized C4 {args.start} start states)",
        "config": {"workload": workload,
                   "n": n, "scenarios_per_gpu": B, "hl_every": 10, "dt": 1e-3, "parallelism": f"scenario-sharded x{world}"},
        "stats": {"agent_qp_solves": qps_all, "ipm_iters": ipm_all, "mean_ipm_iters_per_qp": ipm_all / max(qps_all, 1),
                  "mean_active_rows": row_all / max(ipm_all, 1),
                  "mean_admm_iters": float(np.mean(all_metrics[:, 0])), "collisions_last_step": int(all_metrics[:, 2].sum()),
                  "hl_kernel_ms_per_step": launch_ms, "env_classes": classes},
        "roofline": {"bound": "fp64-valu", "achieved": achieved_tflops, "peak": FP64_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved_tflops / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "traffic_source": traffic_src, "kernel": kernel, "launch_ms": kernel_ms,
                     "flops_per_launch": flops_launch,
                     "flop_model": f"{FLOPS_FIXED:.0f} + {FLOPS_PER_ROW:.0f} x active rows per IPM iteration"},
    }
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(n, args.cpu_sample_s, args.start)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
