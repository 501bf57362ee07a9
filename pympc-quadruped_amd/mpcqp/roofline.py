"""Algorithmic work per QP and MI355X peaks (MI355X_MICROARCH.md).

The figure behind ``roofline.achieved`` is the condensed-dense algorithmic flop
count of one robot's formulate + solve, with n = free GRF variables after the
exact swing elimination (3 x #stance foot-steps) and K = executed active-set
iterations:

  F = 2 n^2 13N            H = Su^T (Qbar Su)           (mpc.py:232)
    + 2 13N 13 + 2 13N n   g = Su^T Qbar (Sx x0 - xref)  (mpc.py:233)
    + N 2 13^3             powers of A                   (mpc.py:213-215)
    + N(N+1)/2 2 13 13 12  Toeplitz blocks A^k B_d       (mpc.py:228-230)
    + n^3 / 3              factorisation
    + K (2 n^2 + 624 N)    per-iteration solves + constraint products

The engine computes H in far fewer flops (Toeplitz/nilpotent structure), so
F is the problem's work, not the kernel's instruction count; the kernel's own
executed float64 flops are reported separately by ``executed_flops``.
"""

PEAK_FP64_TFLOPS = 78.6     # vector FP64 (spec), gfx950
PEAK_FP32_TFLOPS = 157.3    # vector / MFMA FP32 (spec)
PEAK_HBM_GBS = 8000.0       # HBM3E (spec)


def algorithmic_flops(N, n, K):
    return (2 * n * n * 13 * N + 2 * 13 * N * 13 + 2 * 13 * N * n + N * 2 * 13 ** 3
            + N * (N + 1) // 2 * 2 * 13 * 13 * 12 + n ** 3 / 3.0 + K * (2 * n * n + 624 * N))


def executed_flops(N, n, K, q_mean=None):
    """float64 flops the kernel executes: Y/T/H build, sweep inverse, GI iterations."""
    q = n / 2.0 if q_mean is None else q_mean
    build = 9 * 144 * 13 * 2 + 3 * N * 12 * 13 * 2 + n * n * 9 * 2 + n * 3 * N * 2
    sweep = 2.0 * n ** 3
    iters = K * (2 * n * n + 2 * q * q + 4 * q * q + 12 * 6 * n)
    return build + sweep + iters


def input_bytes(N):
    """HBM bytes per QP: x0, xref, contact, feet, robot in; u0, status, iters out."""
    return 4 * (13 + 13 * N + 4 * N + 12 + 16) + 4 * (12 + 2)


def plan_bytes(N, mpc_tick=True, root_layout=False):
    """HBM bytes per robot of one mpcqp_plan launch (include/mpcqp.h).

    in:  quat/pos/omega/vel (52 B) or one root-state row (52 B), R_base (36 B,
         separate layout), body command + yaw rate (32 B float64), planner state
         (48 B), and on an MPC tick height (4 B) + gait record + iteration (40 B);
    out: x0 (52 B), planner state (48 B), and on an MPC tick X_ref (52 N B) and the
         gait table (16 N B)."""
    rd = 52 + (0 if root_layout else 36) + 32 + 48 + (44 if mpc_tick else 0)
    wr = 52 + 48 + ((52 + 16) * N if mpc_tick else 0)
    return rd + wr


def torque_bytes(stance_frac=1.0):
    """HBM bytes per robot of mpcqp_stance_torques: stance mask (16 B) read, and for
    stance legs their 3x3 Jacobian block (36 B) + force (12 B) read, torques (12 B)
    written."""
    return 16 + stance_frac * 4 * (36 + 12 + 12)
