"""CPU oracle, part 1: dtype-faithful NumPy restatement of the reference's
QP formulation (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product path (``mpcqp``) never imports it.

Each function restates one step of ``ModelPredictiveController._solve_mpc``
(``/root/reference/linear_mpc/mpc.py``) with the same layouts and the same
NumPy dtype promotions, so that H, g, C, lb, ub come out equal to what the
reference builds on the same inputs (pinned against fixtures produced by the
reference's own functions: ``tests/golden/make_golden.py``).

Layouts:
  x    = [roll, pitch, yaw, px, py, pz, wx, wy, wz, vx, vy, vz, -g]   (13,)
  xref[13*i + s] is the reference of x_{i+1}                           (13N,)
  contact[4*i + leg], legs FL, FR, RL, RR (1 = stance)                 (4N,)
  U[12*i + 3*leg + axis] = world-frame ground reaction force           (12N,)
  C row 5*(4*i + leg) + r                                              (20N, 12N)
"""
import numpy as np
from scipy.linalg import expm

NUM_STATE = 13
NUM_INPUT = 12

# LinearMpcConfig (config/linear_mpc_configs.py:4-24)
DT_MPC = 0.05            # hard-coded self.dt in mpc.py:38 (not dt_mpc of the config)
GRAVITY = 9.81           # linear_mpc_configs.py:13
MU = 0.7                 # linear_mpc_configs.py:15
Q_DIAG = np.array([5., 5., 10., 10., 10., 50., 0.01, 0.01, 0.2, 0.2, 0.2, 0.2, 0.])  # :19
R_DIAG = np.full(12, 1e-5)                                                          # :20


def make_com_inertial_matrix(ixx, ixy, ixz, iyy, iyz, izz):
    """utils/dynamics.py:3-18 -- symmetric 3x3 inertia, float32."""
    return np.array([[ixx, ixy, ixz], [ixy, iyy, iyz], [ixz, iyz, izz]], dtype=np.float32)


# RobotConfig subclasses (config/robot_configs.py:44-79)
ROBOTS = {
    "aliengo": dict(
        mass=9.042, height=0.38, fz_max=500.0,
        inertia=make_com_inertial_matrix(0.033260231, -0.000451628, 0.000487603,
                                         0.16117211, 4.8356e-05, 0.17460442)),
    "a1": dict(
        mass=4.713, height=0.42, fz_max=500.0,
        # robot_configs.py:73 multiplies the URDF inertia by 10 (float32 * int -> float32)
        inertia=make_com_inertial_matrix(0.01683993, 8.3902e-05, 0.000597679,
                                         0.056579028, 2.5134e-05, 0.064713601) * 10),
}


def skew(v):
    """utils/kinematics.py:166-177 (vec2so3): float64 skew matrix."""
    v = np.asarray(v).reshape(-1)
    s = np.zeros((3, 3))
    s[0, 1], s[0, 2] = -v[2], v[1]
    s[1, 0], s[1, 2] = v[2], -v[0]
    s[2, 0], s[2, 1] = -v[1], v[0]
    return s


def quat_to_zyx(q):
    """utils/kinematics.py:40-49: quaternion (w, x, y, z) -> [roll, pitch, yaw]."""
    import math
    w, x, y, z = (float(c) for c in q)
    roll = math.atan2(2 * (w * x + y * z), 1 - 2 * (x * x + y * y))
    pitch = math.asin(2 * (w * y - z * x))
    yaw = math.atan2(2 * (w * z + x * y), 1 - 2 * (y * y + z * z))
    return [roll, pitch, yaw]


def continuous_model(yaw, inertia_body, mass, feet):
    """mpc.py:173-192 -- A_c (13x13), B_c (13x12), both float32.

    R_z is built in float64 then stored float32 (mpc.py:178-180); the world
    inertia product and its inverse run in float32 (mpc.py:182, :189); the
    skew matrix is float64 so inv(I_w) @ [r]x is float64, rounded on store.
    """
    A = np.zeros((NUM_STATE, NUM_STATE), dtype=np.float32)
    B = np.zeros((NUM_STATE, NUM_INPUT), dtype=np.float32)
    c, s = np.cos(yaw), np.sin(yaw)
    Rz = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]], dtype=np.float32)
    I_world = Rz @ inertia_body @ Rz.T
    A[0:3, 6:9] = Rz.T
    A[3:6, 9:12] = np.eye(3, dtype=np.float32)
    A[11, 12] = 1.0
    I_inv = np.linalg.inv(I_world)
    for leg in range(4):
        B[6:9, 3 * leg:3 * leg + 3] = I_inv @ skew(feet[leg])
        B[9:12, 3 * leg:3 * leg + 3] = np.eye(3, dtype=np.float32) / mass
    return A, B


def discretize(A, B, dt=DT_MPC):
    """mpc.py:194-208 -- expm of the 25x25 float32 block matrix."""
    n, m = NUM_STATE, NUM_INPUT
    M = np.zeros((n + m, n + m), dtype=np.float32)
    M[:n, :n] = A * dt
    M[:n, n:] = B * dt
    E = expm(M)
    return E[:n, :n], E[:n, n:]


def condensed_cost(Ad, Bd, x0, xref, horizon, q_diag=Q_DIAG, r_diag=R_DIAG):
    """mpc.py:211-235 -- H = 2(Su^T Qbar Su + Rbar), g = 2 Su^T Qbar (Sx x0 - xref).

    Powers of A and the Toeplitz blocks of Su are float32 (mpc.py:213-230);
    Qbar is float64 (mpc.py:50) so H and g come out float64.
    """
    n, m, N = NUM_STATE, NUM_INPUT, horizon
    q = np.asarray(q_diag, dtype=np.float64)   # a diagonal, or the full matrix (mpc.py:50,52)
    r = np.asarray(r_diag, dtype=np.float64)
    Qbar = np.kron(np.identity(N), q if q.ndim == 2 else np.diag(q))
    Rbar = np.kron(np.identity(N), r if r.ndim == 2 else np.diag(r))
    powers = [np.identity(n, dtype=np.float32)]
    for _ in range(N):
        powers.append(powers[-1] @ Ad)
    Sx = np.zeros((n * N, n), dtype=np.float32)
    Su = np.zeros((n * N, m * N), dtype=np.float32)
    blocks = [powers[k] @ Bd for k in range(N)]          # A^k Bd, float32
    for i in range(N):
        Sx[n * i:n * (i + 1)] = powers[i + 1]
        for j in range(i + 1):
            Su[n * i:n * (i + 1), m * j:m * (j + 1)] = blocks[i - j]
    H = 2 * (Su.T @ Qbar @ Su + Rbar)
    g = 2 * Su.T @ Qbar @ (Sx @ x0 - xref)
    return H, g, Su, Sx


def cone_rows(mu, normal=None):
    """Friction-pyramid rows.  normal=None (or e_z) is exactly mpc.py:239-245;
    a unit normal n gives [t1+mu n, -t1+mu n, t2+mu n, -t2+mu n, n] with
    t1 = normalise(e_x - n_x n), t2 = n x t1 (build-only generalisation)."""
    if normal is None or np.array_equal(np.asarray(normal, dtype=np.float64), (0.0, 0.0, 1.0)):
        return np.array([[1, 0, mu], [-1, 0, mu], [0, 1, mu], [0, -1, mu], [0, 0, 1]],
                        dtype=np.float32)
    n = np.asarray(normal, dtype=np.float64)
    n = n / np.linalg.norm(n)
    t1 = np.array([1.0, 0.0, 0.0]) - n[0] * n
    t1 /= np.linalg.norm(t1)
    t2 = np.cross(n, t1)
    return np.array([t1 + mu * n, -t1 + mu * n, t2 + mu * n, -t2 + mu * n, n])


def friction_constraints(contact, horizon, mu=MU, fz_max=500.0, normal=None):
    """mpc.py:237-260 -- C = kron(I_4N, cone), lb = 0, ub = [inf x4, contact*fz_max]."""
    cone = cone_rows(mu, normal)
    N = horizon
    C = np.kron(np.identity(4 * N, dtype=cone.dtype), cone)
    lb = np.zeros(20 * N, dtype=np.float32)
    ub = np.zeros(20 * N, dtype=np.float32)
    for k in range(4 * N):
        ub[5 * k:5 * k + 4] = np.inf
        ub[5 * k + 4] = contact[k] * fz_max
    return C, lb, ub


def formulate(x0, xref, contact, feet, inertia, mass, horizon, mu=MU, fz_max=500.0,
              dt=DT_MPC, yaw=None, normal=None, Q=Q_DIAG, R=R_DIAG):
    """The whole formulation half of mpc.py:262-275 for one robot.

    ``yaw`` defaults to x0[2] (mpc.py:77 stores rpy[2] both in the state and in
    self.yaw, so they agree up to the float32 rounding of the state slot).
    ``Q`` / ``R``: diagonals or full matrices (mpc.py:50,52).
    Returns dict(H, g, C, lb, ub, Ad, Bd, Ac, Bc).
    """
    x0 = np.asarray(x0, dtype=np.float32)
    xref = np.asarray(xref, dtype=np.float32).reshape(-1)
    yaw = float(x0[2]) if yaw is None else yaw
    Ac, Bc = continuous_model(yaw, np.asarray(inertia, dtype=np.float32), mass, feet)
    Ad, Bd = discretize(Ac, Bc, dt)
    H, g, _, _ = condensed_cost(Ad, Bd, x0, xref, horizon, Q, R)
    C, lb, ub = friction_constraints(np.asarray(contact).reshape(-1), horizon, mu, fz_max, normal)
    return dict(H=H, g=g, C=C, lb=lb, ub=ub, Ad=Ad, Bd=Bd, Ac=Ac, Bc=Bc)
