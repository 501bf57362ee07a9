"""mpcqp -- MI355X-native batched convex-MPC QP engine.

Drop-in for the formulate-and-solve hot path of yinghansun/pympc-quadruped
(``ModelPredictiveController._solve_mpc``, linear_mpc/mpc.py:262-290).
"""
from .params import (DT_MPC, GAITS, GRAVITY, MU, Q_DIAG, R_DIAG, ROBOT_PRESETS, ROBOT_STRIDE,
                     pack_robot, robot_from_config)

__all__ = ["LinearMpc", "SolveResult", "DT_MPC", "GAITS", "GRAVITY", "MU", "Q_DIAG", "R_DIAG",
           "ROBOT_PRESETS", "ROBOT_STRIDE", "pack_robot", "robot_from_config"]


def __getattr__(name):
    # torch is imported lazily so that the host-only helpers stay importable without it
    if name in ("LinearMpc", "SolveResult"):
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)
