"""CPU-only checks of the C-ABI boundary: libdat.so loads (no GPU needed to load) and exports
every function include/dat.h declares; the Python layout mirror agrees with dat_layout.h."""

import ctypes
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "dat.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(dat_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    from distributed_aerial_transportation_amd import _lib

    _lib.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    names = _declared()
    assert len(names) >= 19
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) <= set(_lib.EXPORTS), set(names) - set(_lib.EXPORTS)


def test_last_error_without_gpu_is_a_clean_error():
    from distributed_aerial_transportation_amd import _lib

    lib = _lib.lib()
    cfg = _lib.Config()
    lib.dat_default_config(cfg)
    cfg.n = 2  # invalid: rejected before touching a device
    h = _lib.H()
    assert lib.dat_create(cfg, h) < 0
    assert b"n must be" in lib.dat_last_error()


def test_layout_mirror():
    from distributed_aerial_transportation_amd import layout

    assert layout.param_size(3) == 41 + 27 * 3
    assert layout.state_size(6) == 12 * 6 + 18
    assert layout.p_off("FEQ", 6) == 41 + 36
    assert layout.NENV == 10 and abs(layout.GRAVITY - 9.80665) < 1e-15


def test_pack_roundtrip_and_params_match_oracle():
    from distributed_aerial_transportation_amd import layout, scenarios, system
    from oracle import model as om
    from oracle import scenarios as osc

    for n in (3, 6, 16):
        p, col, s = scenarios.rqp_setup(n)
        blk = system.pack_params(p, col)
        po = osc.params(n)
        P = layout.P
        assert blk[P["MT"]] == po.mT
        np.testing.assert_allclose(blk[P["JTI"] : P["JTI"] + 9], po.JT_inv.reshape(-1), rtol=1e-15)
        feq = blk[layout.p_off("FEQ", n) : layout.p_off("FEQ", n) + 3 * n].reshape(n, 3).T
        np.testing.assert_allclose(feq, om.equilibrium_forces(po), rtol=1e-13, atol=1e-13)
        assert blk[P["COLR"]] == osc.col_radius(n)
        x = system.pack_state(s)
        s2 = system.RQPState.unpack(x, n)
        for a in ("R", "w", "xl", "vl", "Rl", "wl"):
            np.testing.assert_array_equal(getattr(s, a), getattr(s2, a))
