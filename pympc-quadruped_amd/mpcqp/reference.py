"""Reference-trajectory generation -- the hot path's immediate caller.

Restates, per controller and batched over robots, the stateful pieces of
``ModelPredictiveController`` that produce X_ref for ``_solve_mpc``:

  update_mpc_if_needed   mpc.py:81-92   desired x/y integration, desired yaw
  generate_reference_trajectory  mpc.py:110-170  position clamp, roll/pitch
                                 compensation, horizon integration of yaw/x/y

All state arrays are float64 of shape [B]; X_ref is float32 [B, N*13] exactly
as the reference stores it (mpc.py:154).
"""
import numpy as np

STATE_DIM = 13


class ReferenceTrajectory:
    """Batched desired-pose integrator + reference trajectory (mpc.py:81-170)."""

    def __init__(self, horizon, height, batch=1, dt=0.05, dt_control=0.001, gravity=9.81,
                 max_pos_error=0.1):
        self.N = int(horizon)
        self.B = int(batch)
        self.dt = dt                      # mpc.py:38
        self.dt_control = dt_control      # linear_mpc_configs.py:6
        self.gravity = gravity
        self.height = np.broadcast_to(np.asarray(height, dtype=np.float64), (self.B,)).copy()
        self.max_pos_error = max_pos_error   # mpc.py:121
        self.first_run = np.ones(self.B, dtype=bool)
        self.xpos_des = np.zeros(self.B)
        self.ypos_des = np.zeros(self.B)
        self.yaw_des = np.zeros(self.B)
        self.roll_init = np.zeros(self.B)
        self.pitch_init = np.zeros(self.B)

    def integrate_desired(self, yaw, vel_world, yaw_rate):
        """mpc.py:84-92: first tick latches (0, 0, yaw); later ticks integrate."""
        yaw = np.broadcast_to(np.asarray(yaw, dtype=np.float64), (self.B,))
        v = np.asarray(vel_world, dtype=np.float64).reshape(self.B, -1)
        rate = np.broadcast_to(np.asarray(yaw_rate, dtype=np.float64), (self.B,))
        first = self.first_run
        self.xpos_des = np.where(first, 0.0, self.xpos_des + self.dt_control * v[:, 0])
        self.ypos_des = np.where(first, 0.0, self.ypos_des + self.dt_control * v[:, 1])
        self.yaw_des = np.where(first, yaw, yaw + self.dt_control * rate)
        self.first_run = np.zeros(self.B, dtype=bool)

    def trajectory(self, x0, vel_world, yaw_rate):
        """mpc.py:110-170 for every robot; updates the clamp and compensation state."""
        x0 = np.asarray(x0, dtype=np.float32).reshape(self.B, STATE_DIM)
        v = np.asarray(vel_world, dtype=np.float64).reshape(self.B, -1)
        rate = np.broadcast_to(np.asarray(yaw_rate, dtype=np.float64), (self.B,))
        px, py = x0[:, 3].astype(np.float64), x0[:, 4].astype(np.float64)
        e = self.max_pos_error
        cx = np.clip(self.xpos_des, px - e, px + e)            # mpc.py:129-132
        cy = np.clip(self.ypos_des, py - e, py + e)            # mpc.py:134-137
        self.xpos_des, self.ypos_des = cx, cy                  # mpc.py:139-140
        vx, vy = x0[:, 9].astype(np.float64), x0[:, 10].astype(np.float64)
        roll, pitch = x0[:, 0].astype(np.float64), x0[:, 1].astype(np.float64)
        with np.errstate(divide="ignore", invalid="ignore"):
            self.pitch_init = np.where(np.abs(vx) > 0.2, self.pitch_init + self.dt * (0.0 - pitch) / vx,
                                       self.pitch_init)        # mpc.py:143-144
            self.roll_init = np.where(np.abs(vy) > 0.1, self.roll_init + self.dt * (0.0 - roll) / vy,
                                      self.roll_init)          # mpc.py:145-146
        self.roll_init = np.clip(self.roll_init, -0.25, 0.25)  # mpc.py:149-150
        self.pitch_init = np.clip(self.pitch_init, -0.25, 0.25)
        roll_comp = vy * self.roll_init
        pitch_comp = vx * self.pitch_init
        N = self.N
        X = np.zeros((self.B, N, STATE_DIM), dtype=np.float32)
        X[:, :, 0] = roll_comp[:, None]
        X[:, :, 1] = pitch_comp[:, None]
        X[:, :, 5] = self.height[:, None]
        X[:, :, 8] = rate[:, None]
        X[:, :, 9] = v[:, 0:1]
        X[:, :, 10] = v[:, 1:2]
        X[:, :, 12] = -self.gravity
        # yaw/x/y are integrated step by step in float32 storage (mpc.py:165-168)
        X[:, 0, 2] = self.yaw_des
        X[:, 0, 3] = cx
        X[:, 0, 4] = cy
        for i in range(1, N):
            X[:, i, 2] = X[:, i - 1, 2] + self.dt * rate
            X[:, i, 3] = X[:, i - 1, 3] + self.dt * v[:, 0]
            X[:, i, 4] = X[:, i - 1, 4] + self.dt * v[:, 1]
        return X.reshape(self.B, N * STATE_DIM)
