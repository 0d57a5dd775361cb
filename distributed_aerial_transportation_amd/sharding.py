"""Scenario sharding over the GPUs of a node, one process per GPU, and the metric collectives of a sharded
run (kernel K8).

Closed-loop scenarios are independent (example/rqp_example.py:120-131 runs one at a time), so a batch
splits into contiguous scenario ranges, one `BatchedController` per GPU, with no collective inside the
control step.  What crosses GPUs is only the per-scenario metrics the reference keeps in its loop's lists
(min env distance, collision flag, iteration counts: example/rqp_example.py:112-138) and the run's work
counters: `gather_rows` all-gathers per-scenario rows in global scenario order (uneven shards included),
`reduce_values` sums or maxes counters.  Both run over an initialised `torch.distributed` group: RCCL
over xGMI ("nccl", tensors on the rank's GPU) on MI355X, gloo on CPU in the tests.

    lo, count = shard_range(rank, world, total)
    eng = BatchedController("cadmm", n, count, params, device=local_rank)
    ...
    rows = gather_rows(np.stack([r.iters, r.min_env_dist, r.collision], 1), device=f"cuda:{local_rank}")
"""

from __future__ import annotations

import numpy as np


def shard_range(rank: int, world: int, total: int) -> tuple[int, int]:
    """(first scenario id, count) of `rank`'s contiguous share of `total` scenarios; the first
    total % world ranks take one more."""
    if not (0 <= rank < world) or total < 0:
        raise ValueError(f"shard_range: rank {rank} of {world}, total {total}")
    base, extra = divmod(total, world)
    return rank * base + min(rank, extra), base + (1 if rank < extra else 0)


def _dist():
    import torch.distributed as dist

    if not dist.is_initialized():
        raise RuntimeError("sharding: torch.distributed is not initialised (one process per GPU)")
    return dist


def gather_rows(local: np.ndarray, device="cpu", group=None) -> np.ndarray:
    """All-gather the rows of every rank's `local` (count_r x k float64) into one (sum count_r) x k array
    in rank order, i.e. global scenario order for `shard_range` shards.  Shards may differ in length:
    the row counts are exchanged first and the shards padded to the longest."""
    import torch

    dist = _dist()
    world = dist.get_world_size(group)
    local = np.ascontiguousarray(local, dtype=np.float64)
    if local.ndim != 2:
        raise ValueError("gather_rows: local must be 2-D (rows x columns)")
    cnt = torch.tensor([local.shape[0]], dtype=torch.int64, device=device)
    counts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    buf = torch.zeros((m, local.shape[1]), dtype=torch.float64, device=device)
    if local.shape[0]:
        buf[: local.shape[0]] = torch.from_numpy(local).to(device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return np.concatenate([p[:c].cpu().numpy() for p, c in zip(parts, counts)], axis=0)


def reduce_values(values, op: str = "sum", device="cpu", group=None) -> np.ndarray:
    """Element-wise sum or max over ranks of a float64 vector (work counters, elapsed times)."""
    import torch

    dist = _dist()
    if op not in ("sum", "max"):
        raise ValueError("reduce_values: op is 'sum' or 'max'")
    t = torch.tensor(np.asarray(values, dtype=np.float64), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX, group=group)
    return t.cpu().numpy()
