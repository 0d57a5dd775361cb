"""Full-size C4 (the bench's own workload): the 65,536 path-start scenarios of bench.py (n = 6
C-ADMM, seeded forests 0..63) for 3 HL steps through the production closed loop (dat_closed_loop: device
desired acceleration -> k_env_class -> k_cadmm / k_cadmm_rob -> 10 rollout steps), and the per-GPU shard of
the 8-GPU split (8,192 scenarios) on 4 sub-batch streams as bench.py runs it (auto_sub_batches).

Size-independent properties (the oracle cannot run 65,536 scenarios):
* every state finite, every ADMM count in [1, max_iter + 1], no collision, no agent QP accepted beyond
  Clarabel's 1e-8;
* a scenario's results do not depend on the batch it runs in, its workgroup slot or the stream: the
  8,192-scenario run on 4 streams equals the first 8,192 scenarios of the 65,536-scenario run bitwise
  (states after 3 HL steps, ADMM counts).  The two runs group differently: 10 scenario slots per k_cadmm
  wavefront at 65,536, 8 per wavefront in each 2,048-scenario sub-batch (cadmm_slots), and G selects the
  row-state instantiation of each env class (cadmm_row_mode: registers or LDS);
* the first 64 scenarios equal the CPU restatement (cpu_baseline/dat_cpu.hip: the same per-scenario loop
  and per-lane code, compiled for the host; tests/test_cpu_baseline.py pins it against the reference's own
  closed loop) to 1e-9 in the states."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, STEPS = 6, 3


def _run(sf, st, forests, subs):
    from distributed_aerial_transportation_amd import BatchedController, scenarios

    B = len(sf)
    eng = BatchedController("cadmm", N, B, scenarios.params_block(N))
    eng.set_forests(forests, sf)
    eng.set_state(st, np.zeros(B, dtype=np.int32))
    if subs > 1:
        eng.set_sub_batches(subs)
    eng.closed_loop(STEPS)
    eng.synchronize()
    x, _ = eng.get_state()
    r = eng.control(None, None)  # the 4th step's outputs (ADMM counts, statuses, env distances)
    return x, r, eng.work()


def test_gpu_c4_fullsize_properties():
    import bench
    import cpu_baseline as cb
    from distributed_aerial_transportation_amd import scenarios

    sf, st, forests = bench.bench_states(N, 65536, 0, 1, 64, "path", None)
    x_full, r_full, w_full = _run(sf, st, forests, 1)
    assert np.all(np.isfinite(x_full))
    assert np.all((r_full.iters >= 1) & (r_full.iters <= 101))
    assert not np.any(r_full.collision)
    assert w_full["inband_beyond_clarabel_tol"] == 0
    S = 8192
    x_sub, r_sub, w_sub = _run(sf[:S], st[:S], forests, bench.auto_sub_batches(S))
    assert np.array_equal(x_sub, x_full[:S]), np.argwhere(np.any(x_sub != x_full[:S], axis=1))[:8].ravel()
    assert np.array_equal(r_sub.iters, r_full.iters[:S])
    assert np.array_equal(r_sub.f_des, r_full.f_des[:S])
    # the CPU restatement on the first 64 scenarios
    C = 64
    c = cb.CpuClosedLoop(N, C, scenarios.params_block(N))
    c.set_forests(forests, sf[:C])
    c.set_state(st[:C])
    c.closed_loop(STEPS, threads=min(16, cb.CpuClosedLoop.max_threads()))
    xc, _, _ = c.get()
    c.close()
    err = np.max(np.abs(xc - x_full[:C]) / np.maximum(1.0, np.abs(x_full[:C])))
    print(f"C4 full size: {len(sf)} scenarios x {STEPS} HL steps, {w_full['qp_solves']} agent QPs; 8,192 on "
          f"{bench.auto_sub_batches(S)} streams bitwise equal; CPU restatement (64) max rel state diff {err:.2e}")
    assert err < 1e-9, err
