"""Scenario sharding over the GPUs of a node, one process per GPU, and the metric collectives of a sharded
run (kernel K8).

Closed-loop scenarios are independent (example/rqp_example.py:120-131 runs one at a time), so a batch
splits into contiguous scenario ranges, one `BatchedController` per GPU, with no collective inside the
control step.  What crosses GPUs is only the per-scenario metrics the reference keeps in its loop's lists
(min env distance, collision flag, iteration counts: example/rqp_example.py:112-138) and the run's work
counters: `gather_rows` all-gathers per-scenario rows in global scenario order (uneven shards included),
`reduce_values` sums or maxes counters.  Both run over a `Comm`: RCCL over xGMI through libdat.so's C-ABI
(dat_comm_*, no PyTorch in the rank processes).

    comm = Comm.from_env()                      # RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* of the launcher
    lo, count = shard_range(comm.rank, comm.world, total)
    eng = BatchedController("cadmm", n, count, params, device=comm.device)
    ...
    rows = gather_rows(np.stack([r.iters, r.min_env_dist, r.collision], 1), comm)
"""

from __future__ import annotations

import ctypes
import os
import time

import numpy as np

from . import _lib as L


def shard_range(rank: int, world: int, total: int) -> tuple[int, int]:
    """(first scenario id, count) of `rank`'s contiguous share of `total` scenarios; the first
    total % world ranks take one more."""
    if not (0 <= rank < world) or total < 0:
        raise ValueError(f"shard_range: rank {rank} of {world}, total {total}")
    base, extra = divmod(total, world)
    return rank * base + min(rank, extra), base + (1 if rank < extra else 0)


ID_BYTES = 128  # DAT_COMM_ID_BYTES


def _ccheck(rc: int) -> None:
    if rc != 0:
        raise L.DatError(L.lib().dat_comm_last_error().decode())


class Comm:
    """RCCL communicator of a sharded run, one process per GPU (libdat.so: dat_comm_create / allgather /
    allreduce / barrier).  Host numpy buffers in and out."""

    def __init__(self, device: int, world: int, rank: int, uid: bytes) -> None:
        if len(uid) != ID_BYTES:
            raise ValueError("Comm: the RCCL unique id has 128 bytes")
        self.device, self.world, self.rank = int(device), int(world), int(rank)
        self._lib = L.lib()
        self._h = L.H()
        buf = (ctypes.c_uint8 * ID_BYTES).from_buffer_copy(uid)
        _ccheck(self._lib.dat_comm_create(self.device, self.world, self.rank, buf, ctypes.byref(self._h)))

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * ID_BYTES)()
        _ccheck(L.lib().dat_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def from_env(cls, device: int | None = None, timeout_s: float = 120.0) -> "Comm":
        """The communicator of the launcher's process group (torch.distributed.run or bench.py's own spawn):
        RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT.  Rank 0 creates the RCCL id and hands it to
        the other ranks through a file keyed by the rendezvous address and the launcher's process id (all ranks
        are its children), written atomically; the file is removed once the communicator exists."""
        rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
        dev = int(os.environ.get("LOCAL_RANK", "0")) if device is None else int(device)
        if world == 1:
            return cls(dev, 1, 0, cls.unique_id())
        key = f"{os.environ.get('MASTER_ADDR', 'local')}_{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}"
        path = os.path.join(os.environ.get("DAT_COMM_DIR", "/tmp"), f"dat_comm_{key}.id")
        if rank == 0:
            uid = cls.unique_id()
            tmp = f"{path}.{os.getpid()}"
            with open(tmp, "wb") as f:
                f.write(uid)
            os.replace(tmp, path)
        else:
            t0 = time.monotonic()
            while not os.path.exists(path):
                if time.monotonic() - t0 > timeout_s:
                    raise TimeoutError(f"Comm.from_env: rank {rank} found no RCCL id at {path}")
                time.sleep(0.01)
            with open(path, "rb") as f:
                uid = f.read()
        comm = cls(dev, world, rank, uid)  # collective: returns once every rank has joined
        if rank == 0:
            try:
                os.remove(path)
            except OSError:
                pass
        return comm

    def allgather(self, x) -> np.ndarray:
        """(world, count) array of every rank's float64 vector x (count values each), rank order."""
        x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
        out = np.empty((self.world, x.size))
        _ccheck(self._lib.dat_comm_allgather(self._h, L.ptr(x), x.size, L.ptr(out)))
        return out

    def allreduce(self, x, op: str = "sum") -> np.ndarray:
        if op not in ("sum", "max"):
            raise ValueError("allreduce: op is 'sum' or 'max'")
        y = np.array(x, dtype=np.float64).reshape(-1)
        _ccheck(self._lib.dat_comm_allreduce(self._h, L.ptr(y), y.size, 0 if op == "sum" else 1))
        return y.reshape(np.shape(x))

    def barrier(self) -> None:
        _ccheck(self._lib.dat_comm_barrier(self._h))

    def close(self) -> None:
        if self._h:
            self._lib.dat_comm_destroy(self._h)
            self._h = L.H()

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:  # noqa: BLE001 (interpreter shutdown)
            pass


def gather_rows(local: np.ndarray, comm) -> np.ndarray:
    """All-gather the rows of every rank's `local` (count_r x k float64) into one (sum count_r) x k array
    in rank order, i.e. global scenario order for `shard_range` shards.  Shards may differ in length:
    the row counts are exchanged first and the shards padded to the longest."""
    local = np.ascontiguousarray(local, dtype=np.float64)
    if local.ndim != 2:
        raise ValueError("gather_rows: local must be 2-D (rows x columns)")
    counts = comm.allgather(np.array([local.shape[0]], dtype=np.float64))[:, 0].astype(int)
    m, k = int(counts.max()) if counts.size else 0, local.shape[1]
    buf = np.zeros((m, k))
    buf[: local.shape[0]] = local
    parts = comm.allgather(buf.reshape(-1)).reshape(comm.world, m, k)
    return np.concatenate([parts[r, : counts[r]] for r in range(comm.world)], axis=0)


def reduce_values(values, op: str, comm) -> np.ndarray:
    """Element-wise sum or max over ranks of a float64 vector (work counters, elapsed times)."""
    if op not in ("sum", "max"):
        raise ValueError("reduce_values: op is 'sum' or 'max'")
    return comm.allreduce(np.asarray(values, dtype=np.float64), op)
