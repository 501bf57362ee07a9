"""CPU restatement of the hot path's callers -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker of the HIP planner (mpcqp_plan /
mpcqp_stance_torques); the product path never calls it.

Pinned against the reference's own outputs: tests/golden/reftraj.npz,
gait_N*.npz and planner.npz are produced by the reference's functions
(tests/golden/make_golden.py) and tests/test_oracle.py checks this module
against them.

Numerics restate the reference under its pinned NumPy 1.24 (requirements.txt:50):
Python floats and scalar-with-scalar NumPy arithmetic are float64, the state
and X_ref arrays are float32, and quat2ZYXangle / quat2matrix on a float32
quaternion compute their products and sums in float32 scalars.  (The fixtures
were generated under NumPy 2.2, whose NEP 50 rules keep a few of those float64
steps in float32; the two agree to ~1e-7 and the tests say so.)
"""
import math

import numpy as np

NX = 13

# gait.py:16-22 (bound: the commented definition at gait.py:20)
GAITS = {
    "standing": (16, (0, 0, 0, 0), (16, 16, 16, 16)),
    "trot16": (16, (0, 8, 8, 0), (8, 8, 8, 8)),
    "trot10": (10, (0, 5, 5, 0), (5, 5, 5, 5)),
    "jump16": (16, (0, 0, 0, 0), (4, 4, 4, 4)),
    "bound8": (8, (4, 4, 0, 0), (4, 4, 4, 4)),
    "pace16": (16, (8, 0, 8, 0), (8, 8, 8, 8)),
    "pace10": (10, (5, 0, 5, 0), (5, 5, 5, 5)),
}


def quat2zyx(q):
    """utils/kinematics.py:40-49 on a float32 (w, x, y, z) quaternion -> [roll, pitch, yaw]."""
    w, x, y, z = (np.float32(v) for v in np.asarray(q, dtype=np.float32).reshape(4))
    two, one = np.float32(2), np.float32(1)
    roll = math.atan2(float(two * (w * x + y * z)), float(one - two * (x * x + y * y)))
    s = float(two * (w * y - z * x))
    pitch = math.asin(min(max(s, -1.0), 1.0))
    yaw = math.atan2(float(two * (w * z + x * y)), float(one - two * (y * y + z * z)))
    return [roll, pitch, yaw]


def quat2matrix(q):
    """utils/kinematics.py:51-71 on a float32 (w, x, y, z) quaternion, float32 result."""
    w, x, y, z = (np.float32(v) for v in np.asarray(q, dtype=np.float32).reshape(4))
    two = np.float32(2)
    return np.array([
        [w * w + x * x - y * y - z * z, two * (x * y - w * z), two * (w * y + x * z)],
        [two * (w * z + x * y), w * w - x * x + y * y - z * z, two * (y * z - w * x)],
        [two * (x * z - w * y), two * (w * x + y * z), w * w - x * x - y * y + z * z],
    ], dtype=np.float32)


def gait_table(period, offsets, durations, iteration, horizon):
    """gait.py:81-100: (horizon, 4) float32, 1 = stance."""
    t = np.zeros((horizon, 4), dtype=np.float32)
    for i in range(horizon):
        ih = (i + 1 + iteration) % period
        for leg in range(4):
            seg = ih - offsets[leg]
            if seg < 0:
                seg += period
            t[i, leg] = 1.0 if seg < durations[leg] else 0.0
    return t


class PlannerOracle:
    """One robot's ModelPredictiveController planning state (mpc.py:55-170)."""

    def __init__(self, horizon, height, dt=0.05, dt_control=0.001, gravity=9.81, max_pos_error=0.1):
        self.N = int(horizon)
        self.height = float(np.float32(height))
        self.dt, self.dt_control, self.gravity = dt, dt_control, gravity
        self.max_pos_error = max_pos_error         # mpc.py:121
        self.first = True
        self.xpos_des = self.ypos_des = self.yaw_des = 0.0
        self.roll_init = self.pitch_init = 0.0     # mpc.py:58-59
        self.current_state = np.zeros(NX, dtype=np.float32)
        self.yaw = 0.0

    def update_robot_state(self, quat, pos, omega, vel):
        """mpc.py:55-79."""
        rpy = quat2zyx(quat)
        s = self.current_state
        s[0:3] = rpy
        s[3:6] = np.asarray(pos, dtype=np.float32)
        s[6:9] = np.asarray(omega, dtype=np.float32)
        s[9:12] = np.asarray(vel, dtype=np.float32)
        s[12] = -self.gravity
        self.yaw = rpy[2]
        return s.copy()

    def integrate(self, vel_world, yaw_rate):
        """mpc.py:84-92."""
        if self.first:
            self.xpos_des, self.ypos_des, self.yaw_des = 0.0, 0.0, self.yaw
            self.first = False
        else:
            self.xpos_des += self.dt_control * float(vel_world[0])
            self.ypos_des += self.dt_control * float(vel_world[1])
            self.yaw_des = self.yaw + self.dt_control * float(yaw_rate)

    def reference_trajectory(self, vel_world, yaw_rate):
        """mpc.py:110-170 -> X_ref (N, 13) float32."""
        s = self.current_state
        px, py, e = float(s[3]), float(s[4]), self.max_pos_error
        cx, cy = self.xpos_des, self.ypos_des
        if cx - px > e:
            cx = px + e
        if px - cx > e:
            cx = px - e
        if cy - py > e:
            cy = py + e
        if py - cy > e:
            cy = py - e
        self.xpos_des, self.ypos_des = cx, cy
        vx, vy = float(s[9]), float(s[10])
        if abs(vx) > 0.2:
            self.pitch_init += self.dt * (0.0 - float(s[1])) / vx
        if abs(vy) > 0.1:
            self.roll_init += self.dt * (0.0 - float(s[0])) / vy
        self.roll_init = min(max(self.roll_init, -0.25), 0.25)
        self.pitch_init = min(max(self.pitch_init, -0.25), 0.25)
        X = np.zeros((self.N, NX), dtype=np.float32)
        X[:, 0] = vy * self.roll_init
        X[:, 1] = vx * self.pitch_init
        X[0, 2], X[0, 3], X[0, 4] = self.yaw_des, cx, cy
        X[:, 5] = self.height
        X[:, 8] = yaw_rate
        X[:, 9] = vel_world[0]
        X[:, 10] = vel_world[1]
        X[:, 12] = -self.gravity
        for i in range(1, self.N):
            X[i, 2] = float(X[i - 1, 2]) + self.dt * float(yaw_rate)
            X[i, 3] = float(X[i - 1, 3]) + self.dt * float(vel_world[0])
            X[i, 4] = float(X[i - 1, 4]) + self.dt * float(vel_world[1])
        return X

    def state_record(self):
        """The device's MPCQP_PLAN_STRIDE record for this robot."""
        return np.array([self.xpos_des, self.ypos_des, self.yaw_des, self.roll_init, self.pitch_init,
                         0.0 if self.first else 1.0, 0.0, 0.0])


def world_velocity(R, v_body):
    """mpc.py:83: R_base (float32) @ the float64 body-frame command."""
    R = np.asarray(R, dtype=np.float32).astype(np.float64)
    v = np.asarray(v_body, dtype=np.float64)
    return np.array([R[r, 0] * v[0] + R[r, 1] * v[1] + R[r, 2] * v[2] for r in range(3)])


def stance_torques(jac, stance, u0, tau):
    """leg_controller.py:86-89 per robot: tau_leg = Jv_leg^T (-f_leg) for stance legs.

    jac [B,4,3,3] float32, stance [B,4], u0 [B,12]; tau [B,12] is updated in place."""
    jac = np.asarray(jac, dtype=np.float32)
    u0 = np.asarray(u0, dtype=np.float32)
    for b in range(jac.shape[0]):
        for leg in range(4):
            if stance[b][leg] > 0:
                f = u0[b, 3 * leg:3 * leg + 3]
                tau[b, 3 * leg:3 * leg + 3] = jac[b, leg].T @ -f
    return tau
