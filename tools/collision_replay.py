"""Collisions of the sustained C4 loop (bench.py sustained_loop: 65,536 scenarios, 1,000 HL steps) on the GPU:
which scenarios collide and at which step, and a fixture of the earliest ones for the oracle replay
(tests/test_collision_replay.py): each scenario's state `lead` steps before its first collision, and the GPU's own
replay from there with the warm state reset (the replay's start in the oracle as well) -- per step f_des, ADMM
iterations, min env distance and the collision flag.

    python tools/collision_replay.py out.npz [--steps 1000] [--count 4] [--lead 3] [--after 2]   # on the GPU box
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N = 6
B = 65536


def engine(forests, sf, states):
    import bench
    from distributed_aerial_transportation_amd import BatchedController, scenarios

    eng = BatchedController("cadmm", N, len(sf), scenarios.params_block(N))
    eng.set_qp_tolerance(1e-10)
    eng.set_forests(forests, sf)
    eng.reset_warm_start()
    eng.set_state(states, np.zeros(len(sf), dtype=np.int32))
    if len(sf) == B:
        eng.set_sub_batches(bench.auto_sub_batches(B))
    return eng


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--count", type=int, default=4)
    ap.add_argument("--lead", type=int, default=3)
    ap.add_argument("--after", type=int, default=2)
    args = ap.parse_args()
    import bench

    sf, states, forests = bench.bench_states(N, B, 0, 1, 64, "path", None)
    # pass 1: the loop step by step (control, then the 10 low-level steps: one closed-loop HL step), the
    # scenarios' collision flags
    eng = engine(forests, sf, states)
    first = np.full(B, -1)
    hits = np.zeros(B, dtype=np.int64)
    t0 = time.time()
    for k in range(args.steps):
        r = eng.control()
        new = r.collision & (first < 0)
        first[new] = k
        hits += r.collision
        eng.rollout(10)
        if k % 100 == 0:
            print(f"step {k}: {int((first >= 0).sum())} scenarios collided so far ({time.time() - t0:.0f} s)", flush=True)
    eng.close()
    ids = np.flatnonzero(first >= 0)
    print(f"{len(ids)} scenarios collide ({int(hits.sum())} scenario-steps); first collisions at steps "
          f"{sorted(set(first[ids].tolist()))[:20]}", flush=True)
    if len(ids) == 0:
        np.savez_compressed(args.path, ids=ids)
        return
    pick = ids[np.argsort(first[ids], kind="stable")[:args.count]]
    s0 = first[pick] - args.lead
    # pass 2: the same loop (deterministic) up to each picked scenario's start step, its state there
    eng = engine(forests, sf, states)
    st0 = np.zeros((len(pick), states.shape[1]))
    c0 = np.zeros(len(pick), dtype=np.int32)
    for k in range(int(s0.max()) + 1):
        at = np.flatnonzero(s0 == k)
        if len(at):
            st, c = eng.get_state()
            st0[at], c0[at] = st[pick[at]], c[pick[at]]
        r = eng.control()
        eng.rollout(10)
    eng.close()
    # the GPU replay from st0 with the warm state reset
    K = args.lead + 1 + args.after
    eng = engine(forests, sf[pick], st0)
    eng.set_state(st0, c0)
    f = np.zeros((K, len(pick), 3, N))
    it = np.zeros((K, len(pick)), dtype=np.int32)
    md = np.zeros((K, len(pick)))
    col = np.zeros((K, len(pick)), dtype=bool)
    for k in range(K):
        r = eng.control()
        f[k], it[k], md[k], col[k] = r.f_des, r.iters, r.min_env_dist, r.collision
        eng.rollout(10)
    eng.close()
    for q, s in enumerate(pick):
        print(f"scenario {int(s)} (forest {int(sf[s])}): first collision at step {int(first[s])}, {int(hits[s])} "
              f"collided steps; replay from step {int(s0[q])}, warm state reset: collision at replay steps "
              f"{np.flatnonzero(col[:, q]).tolist()}, min dist {md[:, q].round(6).tolist()}, iters {it[:, q].tolist()}",
              flush=True)
    np.savez_compressed(args.path, ids=pick, forest=sf[pick], first=first[pick], hits=hits[pick], s0=s0, st0=st0,
                        c0=c0, f_des=f, iters=it, min_env_dist=md, collision=col, n_collided=len(ids),
                        scenario_steps=int(hits.sum()))


if __name__ == "__main__":
    main()
