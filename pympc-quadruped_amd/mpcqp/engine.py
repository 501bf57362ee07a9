"""Batched convex-MPC QP engine (host side).

``LinearMpc(...).solve(state, xref, contact_schedule, feet=...)`` formulates
and solves B independent reference MPC QPs in one HIP launch and returns the
first-step ground-reaction forces u0[B, 12] -- the batched form of
``ModelPredictiveController._solve_mpc(...)[0:12]``
(/root/reference/linear_mpc/mpc.py:262-290, :99).

torch-ROCm tensors are storage only: inputs are moved (zero-copy when they are
already contiguous float32 tensors on the engine's device) and the compute is
the HIP kernel behind ``libmpcqp.so`` (include/mpcqp.h).  There is no CPU path.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .params import (DT_MPC, Q_DIAG, R_DIAG, ROBOT_PRESETS, ROBOT_STRIDE, pack_robot)


def _weights(W, n, name):
    """(diagonal, full) from a length-n vector or an n x n matrix: ``full`` is the
    row-major float64 matrix when it has off-diagonal entries (mpcqp_set_weights),
    else None (the diagonal fast path; mpc.py:50,52 build Qbar / Rbar by kron)."""
    W = np.asarray(W, dtype=np.float64)
    if W.shape == (n,):
        return W, None
    if W.shape == (n, n):
        if np.any(W - np.diag(np.diag(W)) != 0.0):
            if not np.allclose(W, W.T, rtol=0.0, atol=1e-12 * max(np.abs(W).max(), 1e-300)):
                raise ValueError(f"{name} is not symmetric")
            return np.diag(W).copy(), np.ascontiguousarray(W)
        return np.diag(W).copy(), None
    raise ValueError(f"{name}: expected ({n},) or ({n}, {n}), got {W.shape}")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


class SolveResult:
    """u0[B,12] plus optional U[B,N,12], status[B], iterations[B] (device tensors)."""

    def __init__(self, u0, U, status, iters):
        self.u0, self.U, self.status, self.iterations = u0, U, status, iters


class LinearMpc:
    """Batched reference MPC: one QP per robot, solved on one MI355X.

    Args:
      horizon:  N (LinearMpcConfig.horizon, config/linear_mpc_configs.py:11)
      robot:    default per-robot parameters: a preset name ("a1", "aliengo"),
                a reference RobotConfig class, or a packed [16] record.
      dt:       model step (hard-coded 0.05 in mpc.py:38)
      Q, R:     weights (linear_mpc_configs.py:19-20): [13] / [12] diagonals or full
                symmetric 13 x 13 / 12 x 12 matrices (set_weights)
      device:   torch device of the HIP context (default cuda:0)
      max_iter: active-set iteration cap per robot (0 = engine default)
      max_stance: optional promise of at most this many stance foot-steps per
                robot (lets the engine skip larger capacity classes)
    """

    def __init__(self, horizon=16, robot="aliengo", dt=DT_MPC, Q=Q_DIAG, R=R_DIAG,
                 device="cuda:0", max_iter=0, max_stance=0):
        self.horizon = int(horizon)
        if not 1 <= self.horizon <= _lib.MAX_HORIZON:
            raise ValueError(f"horizon {self.horizon} outside the engine's 1..{_lib.MAX_HORIZON} "
                             "(MPCQP_MAX_HORIZON, include/mpcqp.h)")
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("LinearMpc runs on a HIP device only (no CPU path)")
        self.lib = _lib.load()
        p = _lib.default_params(self.horizon)
        p.dt = float(dt)
        p.max_iter = int(max_iter)
        qd, qf = _weights(Q, 13, "Q")
        rd, rf = _weights(R, 12, "R")
        for i, v in enumerate(qd):
            p.q_diag[i] = float(v)
        for i, v in enumerate(rd):
            p.r_diag[i] = float(v)
        self.params = p
        ctx = ctypes.c_void_p()
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        _lib.check(None, self.lib.mpcqp_create(ctypes.byref(p), int(idx), ctypes.byref(ctx)),
                   "mpcqp_create")
        self._ctx = ctx
        if qf is not None or rf is not None:
            self.set_weights(Q, R)
        self._hint = (0, 0)
        if max_stance:
            self.set_stance_hint(max_stance)
        self.default_robot = self._robot_record(robot)

    def set_weights(self, Q, R):
        """Replace the cost weights (include/mpcqp.h mpcqp_set_weights): diagonals or full
        symmetric matrices (every capacity class takes any symmetric Q and R; a cross-leg R
        runs the interior-point class's 12 x 12 stage-weight instantiations)."""
        qd, qf = _weights(Q, 13, "Q")
        rd, rf = _weights(R, 12, "R")
        qm = np.ascontiguousarray(qf if qf is not None else np.diag(qd), dtype=np.float64)
        rm = np.ascontiguousarray(rf if rf is not None else np.diag(rd), dtype=np.float64)
        _lib.check(self._ctx, self.lib.mpcqp_set_weights(self._ctx, qm.ctypes.data, rm.ctypes.data),
                   "mpcqp_set_weights")
        self.weights = (qm, rm)

    def set_stance_hint(self, max_stance):
        """Promise at most ``max_stance`` stance foot-steps per robot in the following
        solves (0 = no promise): capacity classes above 3 * max_stance variables are
        not launched.  A robot breaking the promise gets MPCQP_STATUS_TOO_LARGE."""
        self.set_stance_range(0, max_stance)

    def set_stance_range(self, min_stance, max_stance):
        """Promise between ``min_stance`` and ``max_stance`` stance foot-steps per robot
        (include/mpcqp.h): only the capacity classes the range can need are launched,
        the first of them directly on the batch (the drop-in passes the exact count)."""
        rng = (int(min_stance), int(max_stance))
        if rng != getattr(self, "_hint", None):
            _lib.check(self._ctx, self.lib.mpcqp_set_stance_range(self._ctx, *rng), "set_stance_range")
            self._hint = rng

    def set_order(self, mode):
        """Dispatch order of the following solves (include/mpcqp.h mpcqp_set_order): 1 (the
        default) deals each launch's robots to workgroups largest predicted solve time first,
        0 keeps the batch order.  Results are bitwise the same either way."""
        _lib.check(self._ctx, self.lib.mpcqp_set_order(self._ctx, int(mode)), "mpcqp_set_order")

    def set_warm_start(self, capacity):
        """Remember each robot's verified active set between solves (include/mpcqp.h
        mpcqp_set_warm_start): robot b of every later solve starts the interior-point class
        (n > 128, e.g. Gait.STANDING at N = 16) from the rows its previous solve had active,
        and runs the interior point only when they fail the KKT check.  For callers that
        solve the same robots tick after tick; results do not depend on it.  ``capacity`` =
        robots remembered (robot indices 0 .. capacity - 1), 0 disables.  Returns the
        engine-owned device memory (uint8 [capacity, WARM_BYTES]); zero it to forget.
        Replacing it releases the previous memory to torch's allocator on the current
        stream: call it between solves issued on that stream."""
        cap = int(capacity)
        if cap < 0:
            raise ValueError("capacity must be >= 0")
        mem = torch.zeros((cap, _lib.WARM_BYTES), dtype=torch.uint8, device=self.device) if cap else None
        _lib.check(self._ctx, self.lib.mpcqp_set_warm_start(self._ctx, mem.data_ptr() if cap else None, cap),
                   "mpcqp_set_warm_start")
        self._warm = mem   # the context holds its pointer: keep it alive
        return mem

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx is not None and ctx.value:
            try:
                self.lib.mpcqp_destroy(ctx)
            except Exception:
                pass
            self._ctx = None

    @staticmethod
    def _robot_record(robot):
        if robot is None:
            return None
        if isinstance(robot, str):
            return pack_robot(ROBOT_PRESETS[robot])
        if hasattr(robot, "mass_base"):
            from .params import robot_from_config
            return robot_from_config(robot)
        rec = np.asarray(robot, dtype=np.float32).reshape(-1)
        if rec.shape[0] != ROBOT_STRIDE:
            raise ValueError(f"robot record must have {ROBOT_STRIDE} entries")
        return rec

    def _dev(self, a, shape, name):
        t = torch.as_tensor(a)
        t = t.to(device=self.device, dtype=torch.float32).contiguous()
        if tuple(t.shape) != tuple(shape):
            try:
                t = t.reshape(shape)
            except RuntimeError:
                raise ValueError(f"{name}: expected shape {shape}, got {tuple(t.shape)}")
        return t

    def solve(self, state, xref, contact_schedule, feet, robot=None, return_all=False, stream=None):
        """Formulate + solve B QPs.

        state:            [B,13] x0 (mpc.py:65-77) -- x0[2] is the yaw of the model
        xref:             [B,N,13] or [B,13N] reference (mpc.py:154-168)
        contact_schedule: [B,N,4] or [B,4N] gait table (gait.py:81-100)
        feet:             [B,4,3] foot positions relative to the CoM, world frame
        robot:            [B,16] per-robot records, or one record / preset for all
        Returns u0 [B,12] (device tensor), or a SolveResult if return_all.
        """
        st = torch.as_tensor(state)
        B = int(st.shape[0]) if st.dim() == 2 else 1
        N = self.horizon
        cur = torch.cuda.current_stream(self.device)
        if stream is None:
            stream = cur
        elif stream != cur:
            # inputs produced (or copied below) on the current stream must be ready
            # before the launch stream reads them
            stream.wait_stream(cur)
        with torch.cuda.stream(stream):
            return self._solve_on(stream, state, xref, contact_schedule, feet, robot, return_all, B, N)

    def _solve_on(self, stream, state, xref, contact_schedule, feet, robot, return_all, B, N):
        x0 = self._dev(state, (B, 13), "state")
        xr = self._dev(xref, (B, N, 13), "xref")
        ct = self._dev(contact_schedule, (B, N, 4), "contact_schedule")
        ft = self._dev(feet, (B, 4, 3), "feet")
        if robot is None:
            if self.default_robot is None:
                raise ValueError("no robot parameters")
            rb = torch.as_tensor(np.tile(self.default_robot, (B, 1)))
        else:
            r = robot if not isinstance(robot, str) and not hasattr(robot, "mass_base") else None
            if r is None:
                rb = torch.as_tensor(np.tile(self._robot_record(robot), (B, 1)))
            else:
                rt = torch.as_tensor(r)
                rb = rt.reshape(1, -1).expand(B, -1) if rt.dim() == 1 else rt
        rb = self._dev(rb, (B, ROBOT_STRIDE), "robot")
        u0 = torch.empty((B, 12), dtype=torch.float32, device=self.device)
        U = torch.empty((B, N, 12), dtype=torch.float32, device=self.device) if return_all else None
        status = torch.empty((B,), dtype=torch.int32, device=self.device)
        iters = torch.empty((B,), dtype=torch.int32, device=self.device)
        code = self.lib.mpcqp_solve(self._ctx, B, _ptr(x0), _ptr(xr), _ptr(ct), _ptr(ft), _ptr(rb),
                                    _ptr(u0), _ptr(U), _ptr(status), _ptr(iters),
                                    ctypes.c_void_p(stream.cuda_stream))
        _lib.check(self._ctx, code, "mpcqp_solve")
        # the caching allocator must not hand these blocks to other streams' work
        # before the launch has finished with them
        for t in (x0, xr, ct, ft, rb, u0, U, status, iters):
            if t is not None and t.numel():
                t.record_stream(stream)
        if return_all:
            return SolveResult(u0, U, status, iters)
        return u0

    def solve_raw(self, B, x0, xref, contact, feet, robot, u0, U=None, status=None, iters=None,
                  stream=None):
        """Zero-overhead launch on preallocated contiguous float32 device tensors."""
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        code = self.lib.mpcqp_solve(self._ctx, int(B), _ptr(x0), _ptr(xref), _ptr(contact),
                                    _ptr(feet), _ptr(robot), _ptr(u0), _ptr(U), _ptr(status),
                                    _ptr(iters), ctypes.c_void_p(stream.cuda_stream))
        _lib.check(self._ctx, code, "mpcqp_solve")

    def bind_solve(self, B, x0, xref, contact, feet, robot, u0, U=None, status=None, iters=None):
        """solve_raw with its device pointers resolved once: returns ``launch(stream)``.
        For callers that reuse the same preallocated buffers every tick (the drop-in
        controller): the per-call cost is then one ctypes call."""
        lib, ctx = self.lib, self._ctx
        args = (ctx, int(B), _ptr(x0), _ptr(xref), _ptr(contact), _ptr(feet), _ptr(robot), _ptr(u0), _ptr(U),
                _ptr(status), _ptr(iters))
        keep = (x0, xref, contact, feet, robot, u0, U, status, iters)   # the pointers' owners stay alive

        def launch(stream):
            _lib.check(ctx, lib.mpcqp_solve(*args, ctypes.c_void_p(stream.cuda_stream)), "mpcqp_solve")
        launch.buffers = keep
        return launch

    # ---- the hot path's callers on the device (include/mpcqp.h) ----

    def set_planner(self, dt_control=0.001, gravity=9.81, max_pos_error=0.1):
        """Planner constants (linear_mpc_configs.py:6,13; mpc.py:121)."""
        _lib.check(self._ctx, self.lib.mpcqp_set_planner(self._ctx, float(dt_control), float(gravity),
                                                         float(max_pos_error)), "mpcqp_set_planner")

    def plan(self, flags, plan_state, x0, vel_body_des, yaw_rate_des, quat=None, pos=None, omega=None,
             vel=None, rot=None, root_states=None, gait=None, iteration=None, height_des=None, xref=None,
             contact=None, stream=None):
        """One control iteration of state packing + pose integration, and on an MPC
        tick the reference trajectory and gait table (mpc.py:55-170, gait.py:76-100).
        ``flags``: True / PLAN_REFERENCE on an MPC tick, PLAN_NO_INTEGRATE to skip the
        integrators (include/mpcqp.h).

        Every argument is a preallocated contiguous device tensor (float32, except
        plan_state / vel_body_des / yaw_rate_des float64 and gait / iteration int32);
        ``root_states`` [B,13] (Isaac Gym layout) replaces quat/pos/omega/vel/rot."""
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        B = int(plan_state.shape[0])
        s = ctypes.c_void_p(stream.cuda_stream)
        if root_states is not None:
            code = self.lib.mpcqp_plan_root_states(
                self._ctx, B, int(flags), _ptr(root_states), _ptr(vel_body_des), _ptr(yaw_rate_des),
                _ptr(gait), _ptr(iteration), _ptr(height_des), _ptr(plan_state), _ptr(x0), _ptr(xref),
                _ptr(contact), s)
        else:
            code = self.lib.mpcqp_plan(
                self._ctx, B, int(flags), _ptr(quat), _ptr(pos), _ptr(omega), _ptr(vel), _ptr(rot),
                _ptr(vel_body_des), _ptr(yaw_rate_des), _ptr(gait), _ptr(iteration), _ptr(height_des),
                _ptr(plan_state), _ptr(x0), _ptr(xref), _ptr(contact), s)
        _lib.check(self._ctx, code, "mpcqp_plan")

    def bind_plan(self, plan_state, x0, vel_body_des, yaw_rate_des, quat, pos, omega, vel, rot, height_des,
                  xref):
        """plan() (split state inputs) with its device pointers resolved once: returns
        ``launch(flags, stream)`` (see bind_solve)."""
        lib, ctx = self.lib, self._ctx
        B = int(plan_state.shape[0])
        head = (_ptr(quat), _ptr(pos), _ptr(omega), _ptr(vel), _ptr(rot), _ptr(vel_body_des), _ptr(yaw_rate_des),
                _ptr(None), _ptr(None), _ptr(height_des), _ptr(plan_state), _ptr(x0), _ptr(xref), _ptr(None))
        keep = (plan_state, x0, vel_body_des, yaw_rate_des, quat, pos, omega, vel, rot, height_des, xref)

        def launch(flags, stream):
            _lib.check(ctx, lib.mpcqp_plan(ctx, B, int(flags), *head, ctypes.c_void_p(stream.cuda_stream)),
                       "mpcqp_plan")
        launch.buffers = keep
        return launch

    def stance_torques(self, jac, stance, u0, tau, stance_stride=4, stream=None):
        """tau = Jv_leg^T (-f_leg) for stance legs (leg_controller.py:86-89).

        jac [B,4,3,3] float32 (each leg's 3x3 Jacobian block), stance [B, >=4]
        (> 0 = stance) read with ``stance_stride``, u0 / tau [B,12]."""
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        B = int(u0.shape[0])
        code = self.lib.mpcqp_stance_torques(self._ctx, B, _ptr(jac), _ptr(stance), int(stance_stride), _ptr(u0),
                                             _ptr(tau), ctypes.c_void_p(stream.cuda_stream))
        _lib.check(self._ctx, code, "mpcqp_stance_torques")
