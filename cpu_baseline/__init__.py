"""CPU baseline for bench.py (SURVEY.md 8(d) "CPU baseline plan"): the C4 closed loop on the host's
cores -- the same per-scenario controller loop and per-lane fp64 code as the GPU kernels, compiled
for the host with OpenMP over scenarios (dat_cpu.hip).  Not part of the product package."""

from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "dat_cpu.hip")
LIB = os.path.join(HERE, "libdat_cpu.so")
CSRC = os.path.join(REPO, "distributed_aerial_transportation_amd", "csrc")
DEPS = [SRC] + [os.path.join(CSRC, f) for f in ("dat_core.hpp", "dat_qp.hpp", "dat_layout.h")]
STAMP = LIB + ".srchash"
D = ctypes.POINTER(ctypes.c_double)
I = ctypes.POINTER(ctypes.c_int)
LL = ctypes.POINTER(ctypes.c_longlong)


def _hash() -> str:
    h = hashlib.sha256()
    for d in DEPS:
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def build(force: bool = False) -> str:
    """hipcc host build, -O3 for x86-64-v3 (AVX2/FMA: the dev container's Xeon and the GPU box's EPYC),
    OpenMP; rebuilt when the sources' content hash changes."""
    want = _hash()
    have = open(STAMP).read().strip() if os.path.exists(STAMP) and os.path.exists(LIB) else None
    if force or have != want:
        subprocess.check_call(["hipcc", "-O3", "-march=x86-64-v3", "-fopenmp", "-std=c++17", "-fPIC", "-shared",
                               "--offload-arch=gfx950", SRC, "-o", LIB])
        with open(STAMP, "w") as f:
            f.write(want + "\n")
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run __graft_entry__.build()")
        L = ctypes.CDLL(LIB)
        L.datcpu_create.restype = ctypes.c_void_p
        L.datcpu_create.argtypes = [ctypes.c_int, ctypes.c_int, D]
        L.datcpu_destroy.argtypes = [ctypes.c_void_p]
        L.datcpu_set_forests.argtypes = [ctypes.c_void_p, ctypes.c_int, I, D, I, D]
        L.datcpu_set_state.argtypes = [ctypes.c_void_p, D]
        L.datcpu_closed_loop.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_double, LL, LL]
        L.datcpu_reset_warm.argtypes = [ctypes.c_void_p]
        L.datcpu_get.argtypes = [ctypes.c_void_p, D, D, I]
        _lib = L
    return _lib


def _p(a, t=D):
    return a.ctypes.data_as(t)


class CpuClosedLoop:
    """B scenarios of the C-ADMM closed loop on the host (forests sorted by x, as on the GPU)."""

    def __init__(self, n: int, batch: int, params: np.ndarray) -> None:
        self.n, self.batch = n, batch
        self._params = np.ascontiguousarray(params, dtype=np.float64)
        self._h = lib().datcpu_create(n, batch, _p(self._params))
        if not self._h:
            raise RuntimeError("datcpu_create failed")

    def close(self) -> None:
        if self._h:
            lib().datcpu_destroy(self._h)
            self._h = None

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def set_forests(self, forests, scenario_forest) -> None:
        from distributed_aerial_transportation_amd.system import pack_mountain

        offs = np.zeros(len(forests) + 1, dtype=np.int32)
        trees = []
        for k, f in enumerate(forests):
            t = f.tree_pos[np.argsort(f.tree_pos[:, 0], kind="stable")]
            trees.append(t)
            offs[k + 1] = offs[k] + t.shape[0]
        self._trees = np.ascontiguousarray(np.concatenate(trees), dtype=np.float64)
        self._offs = offs
        self._mnt = np.ascontiguousarray(np.stack([pack_mountain(f) for f in forests]), dtype=np.float64)
        self._sf = np.ascontiguousarray(scenario_forest, dtype=np.int32)
        assert lib().datcpu_set_forests(self._h, len(forests), _p(self._offs, I), _p(self._trees), _p(self._sf, I),
                                        _p(self._mnt)) == 0

    def set_state(self, states: np.ndarray) -> None:
        st = np.ascontiguousarray(states, dtype=np.float64)
        assert lib().datcpu_set_state(self._h, _p(st)) == 0

    def reset_warm(self) -> None:
        """The constructor's warm state and no step history (dat_reset_warm_start on the GPU)."""
        assert lib().datcpu_reset_warm(self._h) == 0

    def closed_loop(self, hl_steps: int, count: int = None, threads: int = 0, hl_every: int = 10, dt: float = 1e-3,
                    first: int = 0):
        """hl_steps closed-loop periods of scenarios [first, first + count); (agent QPs, IPM iterations)."""
        q, it = ctypes.c_longlong(), ctypes.c_longlong()
        count = self.batch - first if count is None else count
        assert lib().datcpu_closed_loop(self._h, hl_steps, first, count, threads, hl_every, dt, ctypes.byref(q),
                                        ctypes.byref(it)) == 0
        return q.value, it.value

    def get(self):
        st = np.empty((self.batch, 12 * self.n + 18))
        fd = np.empty((self.batch, 3 * self.n))
        it = np.empty(self.batch, dtype=np.int32)
        assert lib().datcpu_get(self._h, _p(st), _p(fd), _p(it, I)) == 0
        return st, fd.reshape(self.batch, self.n, 3).transpose(0, 2, 1), it

    @staticmethod
    def max_threads() -> int:
        return int(lib().datcpu_max_threads())
