"""The C4 stall fixture on the GPU with a debug build that prints the robust kernel's loose agent QPs
(diag variant): per HL step, the packed states before the step, then the device's LOOSE lines.
    DAT_LIB_PATH=build_var/libdat_dbgprint.so python tools/c4_hard_capture.py > gpurun_out/hard_capture.log"""
import sys
import numpy as np
sys.path.insert(0, '/root/repo')
from tests._golden import load
from distributed_aerial_transportation_amd import BatchedController, Forest, scenarios
d = load("ref_c4_hard.npz"); n = 6; J, K = d["f_des"].shape[:2]
eng = BatchedController("cadmm", n, J, scenarios.params_block(n))
eng.set_forests([Forest.seeded(int(s)) for s in d["forest_seed"]], np.arange(J, dtype=np.int32))
eng.set_state(d["x0"], np.zeros(J, dtype=np.int32))
states = []
for k in range(K):
    x, _ = eng.get_state()
    states.append(x)
    print("STEP", k, flush=True)
    r = eng.control(None, None)
    eng.synchronize()
    sys.stdout.flush()
    eng.rollout(10)
np.save('/root/repo/gpurun_out/hard_capture_states.npy', np.array(states))
