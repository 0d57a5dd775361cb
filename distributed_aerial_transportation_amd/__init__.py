"""dat-mi355x: MI355X-native batched agent-QP solver for cooperative payload transport.

Drop-in GPU replacement for the controller hot path of AkshayThiru/distributed-aerial-transportation
(the per-step QPs the centralized / C-ADMM / DD controllers hand to cvxpy + Clarabel), built on
hand-written fp64 HIP kernels for gfx950 behind the C-ABI in include/dat.h.
"""

from . import layout, scenarios, system  # noqa: F401  (host-side data, no GPU needed)
from .env_forest import Forest  # noqa: F401
from .system import RQPCollision, RQPParameters, RQPState, pack_params, pack_state  # noqa: F401
from . import rigid_payload  # noqa: F401  (RPCentralizedController / RPDynamics load libdat.so on use)


def __getattr__(name):
    # controllers load libdat.so lazily so that data-only imports work without a GPU
    if name in ("BatchedController", "RQPCentralizedController", "RQPCADMMController", "RQPDDController",
                "RQPClosedLoop", "SolverStatistics", "StepResult", "RQPCADMMPrimalSolver", "RQPDDPrimalSolver", "RQPLowLevelController"):
        from . import control

        return getattr(control, name)
    raise AttributeError(name)
