"""TEST HARNESS ONLY: the `Comm` interface of distributed_aerial_transportation_amd.sharding (allgather /
allreduce / barrier over host float64 arrays) on a torch.distributed gloo group, so that the sharding and
rank-combination code runs world-size-2/3 on a CPU-only host (tests/test_distributed.py, bench.py --selftest).
The product's communicator is sharding.Comm (RCCL through libdat.so); nothing in the package imports this."""

import numpy as np


class GlooComm:
    def __init__(self):
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("GlooComm: init a gloo process group first")
        self._d = dist
        self.world, self.rank, self.device = dist.get_world_size(), dist.get_rank(), 0

    def allgather(self, x) -> np.ndarray:
        import torch

        t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64).reshape(-1).copy())
        parts = [torch.empty_like(t) for _ in range(self.world)]
        self._d.all_gather(parts, t)
        return np.stack([p.numpy() for p in parts])

    def allreduce(self, x, op: str = "sum") -> np.ndarray:
        import torch

        t = torch.tensor(np.asarray(x, dtype=np.float64))
        self._d.all_reduce(t, op=self._d.ReduceOp.SUM if op == "sum" else self._d.ReduceOp.MAX)
        return t.numpy()

    def barrier(self) -> None:
        self._d.barrier()

    def close(self) -> None:
        pass
