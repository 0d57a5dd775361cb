# IPM initial-point sweep on the CPU (dev tool): builds the C++ C4 closed loop (cpu_baseline/) from a copy of
# its sources with the tuned start's constants (IPM_S0, IPM_Z0 in dat_qp.hpp) replaced, and reports IPM
# iterations per agent QP over warm HL steps.
#   python tools/ipm_init_sweep.py <tag> [S0 Z0]
import sys, os, subprocess, ctypes, time
sys.path.insert(0, '/root/repo')
import numpy as np
import cpu_baseline as cb
from distributed_aerial_transportation_amd import Forest, scenarios
import bench
import re
import shutil
tag = sys.argv[1]
s0, z0 = (sys.argv[2], sys.argv[3]) if len(sys.argv) > 3 else ("0.03", "0.03")
lib = f'/tmp/cb_{tag}.so'
if not os.path.exists(lib):
    src = f'/tmp/cb_{tag}_src'
    shutil.rmtree(src, ignore_errors=True)
    shutil.copytree('/root/repo', src, ignore=shutil.ignore_patterns('.git', 'gpurun_out', 'diag', '*.so', '*.npz'))
    qp = os.path.join(src, 'distributed_aerial_transportation_amd', 'csrc', 'dat_qp.hpp')
    t = open(qp).read()
    t = re.sub(r"constexpr double IPM_S0 = [^,]*, IPM_Z0 = [^;]*;", f"constexpr double IPM_S0 = {s0}, IPM_Z0 = {z0};", t)
    open(qp, 'w').write(t)
    subprocess.check_call(["hipcc", "-O3", "-march=x86-64-v3", "-fopenmp", "-std=c++17", "-fPIC", "-shared",
                           "--offload-arch=gfx950", os.path.join(src, os.path.relpath(cb.SRC, '/root/repo')), "-o", lib])
cb.LIB = lib
n, S, F = 6, 768, 64
scen_forest, seed = bench.shard(0, S, F)
rng = np.random.default_rng(seed)
forests = [Forest.seeded(s) for s in range(F)]
states = scenarios.forest_path_states(n, S, rng, forests, scen_forest)
c = cb.CpuClosedLoop(n, S, scenarios.params_block(n))
c.set_forests(forests, scen_forest)
c.set_state(states)
q0, i0 = c.closed_loop(1, threads=8)
q1, i1 = c.closed_loop(2, threads=8)
t = time.time()
q2, i2 = c.closed_loop(4, threads=8)
st, fd, it = c.get()
np.save(f'/tmp/cb_{tag}_st.npy', st)
print(tag, 'cold it/QP %.3f' % (i0 / q0), 'warm it/QP %.3f' % (i2 / q2), 'QPs', q2, 'admm', it.mean(), '%.1fs' % (time.time() - t))
