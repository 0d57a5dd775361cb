"""Replay captured agent QPs (tools/redo_caps.npz: host-build solves that took the robust redo) through the GPU's
single-QP surface (dat_solve_agent_qp_batch, IPM_FAST_REDO) and compare with the host build's answers."""
import sys
import numpy as np
sys.path.insert(0, '/root/repo')
from distributed_aerial_transportation_amd import BatchedController, Forest, scenarios
d = np.load('/root/repo/tools/redo_caps.npz')
K, n = d['state'].shape[0], 6
eng = BatchedController("cadmm", n, K, scenarios.params_block(n))
eng.set_forests([Forest.seeded(int(d['forest_seed']))], np.zeros(K, dtype=np.int32))
eng.set_state(d['state'], np.zeros(K, dtype=np.int32))
r = eng.solve_agent_qps(np.arange(K), d['i'], d['acc'], lam=d['lam'], rho=d['rho'], f_mean=d['fm'])
w = eng.work()
for k in range(K):
    host = d['f'][k].reshape(n, 3).T
    rel = np.max(np.abs(r['x'][k] - host)) / max(1, np.abs(host).max())
    print(k, 'status gpu', int(r['status'][k]), 'host', int(d['status'][k]), 'iters', int(r['ipm_iters'][k]), 'rel %.2e' % rel)
print(w)
