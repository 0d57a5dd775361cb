"""ctypes loader for the TEST-ONLY host build of the per-lane device functions (see hostsim.hip)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libdat_hostsim.so")
SRC = os.path.join(HERE, "hostsim.hip")
CORE = os.path.join(os.path.dirname(os.path.dirname(HERE)), "distributed_aerial_transportation_amd", "csrc")


def build(force=False):
    deps = [SRC] + [os.path.join(CORE, f) for f in ("dat_core.hpp", "dat_qp.hpp", "dat_layout.h")]
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(d) for d in deps):
        subprocess.check_call(["hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                               SRC, "-o", LIB])
    return LIB


_lib = None
D = ctypes.POINTER(ctypes.c_double)
I = ctypes.POINTER(ctypes.c_int)


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
    return _lib


def p(a):
    return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(D)


def qp_cadmm(prm, n, st, acc, lhs, rhs, i, lam, fbar, rho=1.0):
    f = np.zeros(3 * n)
    it = ctypes.c_int()
    lhs = np.ascontiguousarray(lhs, dtype=np.float64).reshape(-1, 3)
    status = lib().hs_qp_cadmm(p(prm), n, p(st), p(acc), p(lhs), p(rhs), lhs.shape[0], i, p(lam), p(fbar),
                               ctypes.c_double(rho), f.ctypes.data_as(D), ctypes.byref(it))
    return f, status, it.value


def qp_cadmm_ex(prm, n, st, acc, lhs, rhs, i, lam, fbar, rho=1.0, tuned=0):
    """hs_qp_cadmm with the IPM start flag of k_cadmm; returns (f, status, iters, inband)"""
    f = np.zeros(3 * n)
    it, ib = ctypes.c_int(), ctypes.c_int()
    lhs = np.ascontiguousarray(lhs, dtype=np.float64).reshape(-1, 3)
    status = lib().hs_qp_cadmm_ex(p(prm), n, p(st), p(acc), p(lhs), p(rhs), lhs.shape[0], i, p(lam), p(fbar),
                                  ctypes.c_double(rho), int(tuned), f.ctypes.data_as(D), ctypes.byref(it),
                                  ctypes.byref(ib))
    return f, status, it.value, ib.value


def _qp_consts():
    """WREC_SIZE and the tail rule (TAIL_PREV, TAIL_PASS) as dat_qp.hpp defines them"""
    import re

    src = open(os.path.join(CORE, "dat_qp.hpp")).read()
    tp = re.search(r"constexpr int TAIL_PREV = (\d+), TAIL_PASS = (\d+);", src)
    assert tp and "constexpr int WREC_SIZE = 28 + 2 * DAT_MAXROW;" in src
    return 28 + 2 * 13, int(tp.group(1)), int(tp.group(2))


WREC_SIZE, TAIL_PREV, TAIL_PASS = _qp_consts()


def qp_cadmm_warm(prm, n, st, acc, lhs, rhs, i, lam, fbar, rho, wrec, wson=True, tuned=0):
    """hs_qp_cadmm_ex as the tail kernel solves it: the certificate of infeasible rows, the warm-start record wrec
    (WREC_SIZE doubles, updated in place) and, wson, the warm first attempt (wrec[0] = 1) and the stall exit;
    returns (f, status, iters, inband)"""
    f = np.zeros(3 * n)
    it, ib = ctypes.c_int(), ctypes.c_int()
    lhs = np.ascontiguousarray(lhs, dtype=np.float64).reshape(-1, 3)
    assert wrec.dtype == np.float64 and wrec.flags.c_contiguous and wrec.size == WREC_SIZE
    status = lib().hs_qp_cadmm_warm(p(prm), n, p(st), p(acc), p(lhs), p(rhs), lhs.shape[0], i, p(lam), p(fbar),
                                    ctypes.c_double(rho), int(tuned), wrec.ctypes.data_as(D), int(bool(wson)), f.ctypes.data_as(D),
                                    ctypes.byref(it), ctypes.byref(ib))
    return f, status, it.value, ib.value


def last_stiff():
    """the last C-ADMM hostsim solve was redone robustly (its fast attempt was not clean: the GPU hands the
    scenario to the tail there)"""
    return lib().hs_last_stiff()


def last_work():
    """(refinement passes, corrections) of the last hostsim QP solve"""
    r, c = ctypes.c_int(), ctypes.c_int()
    lib().hs_last_work(ctypes.byref(r), ctypes.byref(c))
    return r.value, c.value


def last_diag():
    """(merit, inband, exit reason) of the last hostsim QP solve"""
    m, ib, why = ctypes.c_double(), ctypes.c_int(), ctypes.c_int()
    lib().hs_last_diag(ctypes.byref(m), ctypes.byref(ib), ctypes.byref(why))
    return m.value, ib.value, why.value


def qp_dd(prm, n, st, acc, lhs, rhs, i, c9):
    x = np.zeros(9)
    it = ctypes.c_int()
    lhs = np.ascontiguousarray(lhs, dtype=np.float64).reshape(-1, 3)
    status = lib().hs_qp_dd(p(prm), n, p(st), p(acc), p(lhs), p(rhs), lhs.shape[0], i, p(c9), x.ctypes.data_as(D),
                            ctypes.byref(it))
    return x, status, it.value


def qp_cent(prm, n, st, acc, lhs, rhs):
    f = np.zeros(3 * n)
    it = ctypes.c_int()
    lhs = np.ascontiguousarray(lhs, dtype=np.float64).reshape(-1, 3)
    status = lib().hs_qp_cent(p(prm), n, p(st), p(acc), p(lhs), p(rhs), lhs.shape[0], f.ctypes.data_as(D),
                              ctypes.byref(it))
    return f, status, it.value


def env_rows(prm, n, st, trees, agent, alpha):
    lhs = np.zeros((10, 3))
    rhs = np.zeros(10)
    col = ctypes.c_int()
    md = ctypes.c_double()
    trees = np.asarray(trees, dtype=np.float64)
    # env_rows scans an x-window of x-sorted trees (dat_set_forests sorts each forest the same way)
    trees = np.ascontiguousarray(trees[np.argsort(trees[:, 0], kind="stable")])
    k = lib().hs_env_rows(p(prm), n, p(st), p(trees), trees.shape[0], agent, ctypes.c_double(alpha),
                          lhs.ctypes.data_as(D), rhs.ctypes.data_as(D), ctypes.byref(col), ctypes.byref(md))
    return lhs[:k], rhs[:k], bool(col.value), md.value


def sim_step(prm, n, st, counter, fdes, dt, kind=0):
    st = np.array(st, dtype=np.float64)
    c = ctypes.c_int(counter)
    lib().hs_sim_step_ll(p(prm), n, st.ctypes.data_as(D), ctypes.byref(c), p(fdes), ctypes.c_double(dt), int(kind))
    return st, c.value


def ll_control(R, w, J, fdes, kind=0):
    """one agent's low-level law (ll_control_agent): R, J row-major 3x3 (9), w, fdes (3)"""
    f = ctypes.c_double()
    M = np.zeros(3)
    lib().hs_ll_control_kind(p(R), p(w), p(J), p(fdes), ctypes.byref(f), M.ctypes.data_as(D), int(kind))
    return f.value, M


def rp_step(prm, n, st, counter, f, dt):
    """rigid-payload step (rp_step): f (3n) agent-major"""
    st = np.array(st, dtype=np.float64)
    c = ctypes.c_int(counter)
    lib().hs_rp_step(p(prm), n, st.ctypes.data_as(D), ctypes.byref(c), p(f), ctypes.c_double(dt))
    return st, c.value
