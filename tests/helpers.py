"""Shared test helpers: oracle solutions for synthetic batches (CPU, float64)."""
import numpy as np

from oracle import formulation as F
from oracle import qp as QP


def oracle_solution(batch, b, horizon, Q=F.Q_DIAG, R=F.R_DIAG):
    """Reference-faithful formulation + exact QP optimum for robot b of a batch
    (``Q`` / ``R``: diagonals or full matrices, mpc.py:50,52)."""
    x0 = batch["x0"][b]
    xref = batch["xref"][b].reshape(-1)
    contact = batch["contact"][b].reshape(-1)
    feet = batch["feet"][b].astype(np.float64)
    rec = batch["robot"][b]
    inertia = np.array([[rec[1], rec[2], rec[3]], [rec[2], rec[4], rec[5]],
                        [rec[3], rec[5], rec[6]]], dtype=np.float32)
    normal = rec[9:12].astype(np.float64)
    o = F.formulate(x0, xref, contact, feet, inertia, float(rec[0]), horizon,
                    mu=float(rec[7]), fz_max=float(rec[8]), normal=normal, Q=Q, R=R)
    x, y, info = QP.solve_qp_dual_active_set(o["H"], o["g"], o["C"], o["lb"], o["ub"])
    return x, o, info


def rel_err_u0(u0, u0_ref):
    """Norm-wise relative error ||u0 - u0*||_inf / max(||u0*||_inf, 1e-3)."""
    return float(np.abs(np.asarray(u0, np.float64) - u0_ref).max() / max(np.abs(u0_ref).max(), 1e-3))
