"""Drop-in ``ModelPredictiveController`` backed by the MI355X engine.

Same module name, class name, constructor and methods as the reference's
``linear_mpc/mpc.py`` (ModelPredictiveController, mpc.py:22-318), so that
``scripts/mujoco_aliengo.py`` and ``scripts/isaacgym_a1.py`` run unchanged after
``sys.path.append('../linear_mpc'); from mpc import ModelPredictiveController``.

What changes underneath: the planner state (desired x / y / yaw integrators,
roll / pitch compensation, mpc.py:84-152) lives on the device and is advanced
by ``mpcqp_plan`` every control iteration; on MPC ticks X_ref is built there
too and ``_solve_mpc`` (mpc.py:262-290) hands (x0, X_ref, gait table, foot
positions, robot parameters) to ``mpcqp_solve`` without a host round trip.
The QP is never built with NumPy/SciPy nor solved with Drake.  Nothing here
imports pydrake, qpsolvers, numba, pinocchio or matplotlib.

Behaviour kept from the reference:
  * dt = 0.05 regardless of the config (mpc.py:38); the horizon is
    read from the given config (mpc.py:39);
  * the solver string is asserted (mpc.py:264); 'drake' and 'qpsolvers' both
    solve the two-sided Drake-branch QP (the reference's qpsolvers branch drops
    lb), 'hip' is accepted as well;
  * an unsuccessful solve (iteration cap) still returns the best iterate
    (mpc.py:284-286 never checks is_success), with a warning; non-finite inputs
    raise (there is no iterate to return);
  * Q and R are taken whole (mpc.py:50,52): full symmetric matrices go to the
    engine's general-weight path (mpcqp_set_weights), diagonal ones to its
    diagonal fast path; an asymmetric weight raises.
"""
import math
import os
import sys
import warnings

import numpy as np

_PKG = os.environ.get("MPCQP_PATH", os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from mpcqp.params import pack_robot  # noqa: E402


def quat2ZYXangle(quat):
    """utils/kinematics.py:40-49 -- (w, x, y, z) -> [roll, pitch, yaw]."""
    q = np.asarray(quat).reshape(-1)
    roll = math.atan2(2 * (q[0] * q[1] + q[2] * q[3]), 1 - 2 * (q[1] ** 2 + q[2] ** 2))
    pitch = math.asin(2 * (q[0] * q[2] - q[3] * q[1]))
    yaw = math.atan2(2 * (q[0] * q[3] + q[1] * q[2]), 1 - 2 * (q[2] ** 2 + q[3] ** 2))
    return [roll, pitch, yaw]


def _weight_matrix(W, n, name):
    """LinearMpcConfig.Q / .R as an n x n float64 matrix (mpc.py:50,52 build Qbar =
    kron(I_N, Q)); a length-n vector is read as the diagonal."""
    W = np.asarray(W, dtype=np.float64)
    if W.shape == (n,):
        return np.diag(W)
    if W.shape != (n, n):
        raise ValueError(f"{name} must be {n}x{n} (or its diagonal), got {W.shape}")
    if np.any(np.abs(W - W.T) > 1e-12 * max(float(np.abs(W).max()), 1e-300)):
        raise ValueError(f"{name} is not symmetric")
    return W.copy()


class ModelPredictiveController():

    def __init__(self, mpc_config, robot_config):
        self.num_state = 13      # mpc.py:26
        self.num_input = 12      # mpc.py:28
        self.is_initialized = False
        self.is_first_run = True
        self._load_parameters(mpc_config, robot_config)
        self._engine = None

    def _load_parameters(self, mpc_config, robot_config):
        """mpc.py:35-52 (Qbar / Rbar become the engine's weights)."""
        self.dt_control = mpc_config.dt_control
        self.iterations_between_mpc = mpc_config.iteration_between_mpc
        self.dt = 0.05
        self.horizon = mpc_config.horizon
        from mpcqp import _lib
        if not 1 <= int(self.horizon) <= _lib.MAX_HORIZON:
            raise ValueError(f"LinearMpcConfig.horizon = {self.horizon}: the MI355X engine supports "
                             f"1..{_lib.MAX_HORIZON} (MPCQP_MAX_HORIZON, include/mpcqp.h)")
        self.mu = mpc_config.friction_coef
        self.fz_max = robot_config.fz_max
        self.gravity = mpc_config.gravity
        self.base_inertia_base = robot_config.base_inertia_base
        self.mass = robot_config.mass_base
        self.com_height_des = robot_config.base_height_des
        self.Q = _weight_matrix(mpc_config.Q, 13, "Q")
        self.R = _weight_matrix(mpc_config.R, 12, "R")
        I = np.asarray(self.base_inertia_base, dtype=np.float32)
        self._robot_record = pack_robot(
            dict(mass=float(self.mass), fz_max=float(self.fz_max), mu=float(self.mu),
                 inertia=np.array([I[0, 0], I[0, 1], I[0, 2], I[1, 1], I[1, 2], I[2, 2]],
                                  dtype=np.float32)))

    def _get_engine(self):
        if self._engine is None:
            import torch
            from mpcqp import LinearMpc
            from mpcqp._lib import PLAN_STRIDE
            e = LinearMpc(horizon=self.horizon, robot=self._robot_record, dt=self.dt,
                          Q=self.Q, R=self.R, device=os.environ.get("MPCQP_DEVICE", "cuda:0"))
            e.set_planner(dt_control=self.dt_control, gravity=self.gravity)
            # one robot solved every MPC tick: start from the previous tick's active set
            # (the interior-point class only; the optimum is checked either way)
            e.set_warm_start(0 if os.environ.get("MPCQP_COLD") else 1)
            d, f32 = e.device, dict(dtype=torch.float32, device=e.device)
            N = self.horizon
            self._dev = dict(
                plan_state=torch.zeros((1, PLAN_STRIDE), dtype=torch.float64, device=d),
                x0=torch.zeros((1, 13), **f32), xref=torch.zeros((1, N, 13), **f32),
                xref_gen=torch.zeros((1, N, 13), **f32),
                height=torch.full((1,), float(self.com_height_des), **f32),
                robot=torch.as_tensor(self._robot_record).reshape(1, -1).to(d),
                u0=torch.zeros((1, 12), **f32),
                # solve outputs in one buffer: U [12N] f32, status and iterations as int32
                # bits -- one device->host copy per MPC tick
                out=torch.zeros((12 * N + 2,), **f32))
            self._dev["U"] = self._dev["out"][:12 * N]
            self._dev["status"] = self._dev["out"][12 * N:12 * N + 1].view(torch.int32)
            self._dev["iters"] = self._dev["out"][12 * N + 1:].view(torch.int32)
            # one host->device upload per control iteration (byte offsets, 8-aligned):
            # [0, 24) v_des body f64[3], [24, 32) yaw rate f64, [32, 120) the planner's
            # float32 state (quat, pos, omega, vel, R_base), [128, ...) on MPC ticks the
            # gait table f32[4N] and the feet f32[12]
            self._up_bytes = 128 + 4 * (4 * N + 12)
            # page-locked staging, two buffers: the upload is an asynchronous DMA that the
            # plan / solve launches queue behind; a buffer is rewritten only after its
            # previous copy has completed (its event)
            self._up_pinned = [torch.zeros((self._up_bytes,), dtype=torch.uint8, pin_memory=True) for _ in range(2)]
            self._up_events = [None, None]
            self._up_slot = 0
            self._up_host = self._up_pinned[0].numpy()
            self._up_dev = torch.zeros((self._up_bytes,), dtype=torch.uint8, device=d)
            self._out_pinned = torch.zeros((12 * N + 2,), dtype=torch.float32, pin_memory=True)
            self._up_pairs = {}     # (slot, lo, nbytes) -> (device slice, pinned slice)
            self._up_views = None   # device views of the upload buffer's fields
            self._plan_fns = {}     # xref buffer name -> bound mpcqp_plan launcher
            self._solve_fns = {}    # (contact, feet, xref) pointers -> bound mpcqp_solve launcher
            self._engine = e
        return self._engine

    def _upload(self, vel_base_des_body, yaw_turn_rate, gait_table=None):
        """Pack the iteration's host inputs (and on MPC ticks the gait table and foot
        positions) into one buffer and copy it to the device in one transfer."""
        import torch
        slot = self._up_slot = self._up_slot ^ 1
        if self._up_events[slot] is not None:
            self._up_events[slot].synchronize()
        h = self._up_host = self._up_pinned[slot].numpy()
        lo, nbytes = 0, 120
        if vel_base_des_body is None:   # gait table and feet only (a direct _solve_mpc call)
            lo = 128
        else:
            rd = self.__robot_data
            h[0:24].view(np.float64)[:] = np.asarray(vel_base_des_body, dtype=np.float64).reshape(3)
            h[24:32].view(np.float64)[0] = float(yaw_turn_rate)
            f = h[32:120].view(np.float32)
            f[0:4] = np.asarray(rd.quat_base, dtype=np.float32).reshape(4)
            f[4:7] = np.asarray(rd.pos_base, dtype=np.float32).reshape(3)
            f[7:10] = np.asarray(rd.ang_vel_base, dtype=np.float32).reshape(3)
            f[10:13] = np.asarray(rd.lin_vel_base, dtype=np.float32).reshape(3)
            f[13:22] = np.asarray(rd.R_base, dtype=np.float32).reshape(9)
        if gait_table is not None:
            nt = 4 * self.horizon
            g = h[128:self._up_bytes].view(np.float32)
            g[:nt] = np.asarray(gait_table, dtype=np.float32).reshape(-1)
            g[nt:nt + 12] = self._feet_host()
            nbytes = self._up_bytes
        # the (device, pinned) slice pair of this byte range and the device views are
        # built once: torch view / slice ops cost microseconds each on the host
        key = (slot, lo, nbytes)
        pair = self._up_pairs.get(key)
        if pair is None:
            pair = self._up_pairs[key] = (self._up_dev[lo:nbytes], self._up_pinned[slot][lo:nbytes])
        pair[0].copy_(pair[1], non_blocking=True)
        ev = self._up_events[slot] = self._up_events[slot] or torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self._up_dev.device))
        v = self._up_views
        if v is None:
            dev = self._up_dev
            fd = dev[32:120].view(torch.float32)
            g = dev[128:self._up_bytes].view(torch.float32)
            v = self._up_views = dict(
                vb=dev[0:24].view(torch.float64).reshape(1, 3), yr=dev[24:32].view(torch.float64),
                quat=fd[0:4], pos=fd[4:7], omega=fd[7:10], vel=fd[10:13], rot=fd[13:22],
                contact=g[:4 * self.horizon].reshape(1, -1), feet=g[4 * self.horizon:].reshape(1, 4, 3))
        if gait_table is not None:
            v = dict(v, stance=int(np.count_nonzero(h[128:128 + 16 * self.horizon].view(np.float32) > 0)))
        return v

    def _feet_host(self):
        return np.asarray([np.asarray(f, dtype=np.float64).reshape(3) for f in self.pos_base_feet],
                          dtype=np.float32).reshape(-1)

    def _plan(self, flags, up, xref_key="xref"):
        """One mpcqp_plan launch on the preallocated buffers (pointers bound once)."""
        import torch
        e = self._get_engine()
        fn = self._plan_fns.get(xref_key)
        if fn is None:
            dv = self._dev
            fn = self._plan_fns[xref_key] = e.bind_plan(
                dv["plan_state"], dv["x0"], up["vb"], up["yr"], up["quat"], up["pos"], up["omega"], up["vel"],
                up["rot"], dv["height"], dv[xref_key])
        fn(flags, torch.cuda.current_stream(e.device))

    def _planner_state(self):
        return self._dev["plan_state"].cpu().numpy()[0]

    @property
    def xpos_base_desired(self):
        return float(self._planner_state()[0])

    @property
    def ypos_base_desired(self):
        return float(self._planner_state()[1])

    @property
    def yaw_desired(self):
        return float(self._planner_state()[2])

    # data: [pos_base, vel_base, quat_base, omega_base, ...]   (mpc.py:54-79)
    def update_robot_state(self, robot_data):
        if not self.is_initialized:
            self.current_state = np.zeros(13, dtype=np.float32)
            self.roll_init = 0.0
            self.pitch_init = 0.0
            self.is_initialized = True
        self.__robot_data = robot_data
        rpy_base = quat2ZYXangle(robot_data.quat_base)
        pos_base = np.array(robot_data.pos_base, dtype=np.float32)
        omega_base = np.array(robot_data.ang_vel_base, dtype=np.float32)
        vel_base = np.array(robot_data.lin_vel_base, dtype=np.float32)
        self.current_state[0:3] = rpy_base
        self.current_state[3:6] = pos_base
        self.current_state[6:9] = omega_base
        self.current_state[9:12] = vel_base
        self.current_state[12] = -self.gravity          # mpc.py:76
        self.yaw = rpy_base[2]
        self.pos_base_feet = robot_data.pos_base_feet   # world frame, relative to the CoM

    def update_mpc_if_needed(self, iter_counter, base_vel_base_des, yaw_turn_rate_des,
                             gait_table, solver='drake', debug=False, iter_debug=None):
        """mpc.py:81-108: integrators on the device every call, a solve on MPC ticks."""
        self._base_vel_base_des = np.asarray(base_vel_base_des, dtype=np.float64).reshape(3)
        self._get_engine()
        if iter_counter % self.iterations_between_mpc == 0:
            assert solver == 'drake' or solver == 'qpsolvers' or solver == 'hip'
            # one upload (state, command, gait table, feet), integrate + reference
            # trajectory in one launch (mpc.py:84-92, :110-170), then the solve
            up = self._upload(self._base_vel_base_des, yaw_turn_rate_des, gait_table)
            self.__contact_forces = self._mpc_tick(up)[0:12]
            self.is_first_run = False
            self._ref_traj_host = None   # ref_traj (mpc.py:97) is read back only when asked for
            if debug and iter_counter == iter_debug:
                warnings.warn("debug CoM-trajectory plot (mpc.py:293-318) is not provided by the engine")
        else:
            self._plan(0, self._upload(self._base_vel_base_des, yaw_turn_rate_des))
            self.is_first_run = False
        return self.__contact_forces[0:12]

    @property
    def ref_traj(self):
        """X_ref of the last MPC tick (mpc.py:96-97), float32 [13N]."""
        if getattr(self, "_ref_traj_host", None) is None:
            self._ref_traj_host = self._dev["xref"].cpu().numpy().reshape(-1)
        return self._ref_traj_host

    def generate_reference_trajectory(self, vel_base_des, yaw_turn_rate):
        """mpc.py:110-170 alone (stateful clamp + roll/pitch compensation), on the device.

        ``vel_base_des`` is the world-frame command as in the reference; it is mapped
        back to the body frame for the planner, which applies R_base itself."""
        from mpcqp._lib import PLAN_NO_INTEGRATE, PLAN_REFERENCE
        R = np.asarray(self.__robot_data.R_base, dtype=np.float64).reshape(3, 3)
        vb = np.linalg.solve(R, np.asarray(vel_base_des, dtype=np.float64).reshape(3))
        # its own X_ref buffer: ref_traj keeps the last MPC tick's (mpc.py:96-97)
        self._get_engine()
        self._plan(PLAN_REFERENCE | PLAN_NO_INTEGRATE, self._upload(vb, yaw_turn_rate), xref_key="xref_gen")
        return self._dev["xref_gen"].cpu().numpy().reshape(-1)

    def _solve_mpc(self, ref_traj, gait_table, solver='drake', debug=False):
        """mpc.py:262-290 -> one engine call; returns U[12N] (float64, like Drake).

        x0 is the device state the planner packed this iteration; ``ref_traj`` may be
        the planner's device X_ref or a host array."""
        assert solver == 'drake' or solver == 'qpsolvers' or solver == 'hip'
        import torch
        e = self._get_engine()
        up = self._upload(None, 0.0, gait_table)
        xr = ref_traj if isinstance(ref_traj, torch.Tensor) else \
            torch.from_numpy(np.asarray(ref_traj, dtype=np.float32).reshape(1, self.horizon, 13)).to(e.device)
        return self._solve_dev(up["contact"], up["feet"], up["stance"], xr.reshape(1, self.horizon, 13))

    def _solve_dev(self, contact, feet, stance, xref=None):
        """The engine call on device buffers: preallocated outputs, one device->host
        copy (into page-locked memory) and one synchronisation for U and the status."""
        import torch
        e = self._engine
        dv = self._dev
        fn = self._solve_fn(contact, feet, stance, xref)
        fn(torch.cuda.current_stream(e.device))
        self._out_pinned.copy_(dv["out"], non_blocking=True)
        torch.cuda.current_stream(dv["out"].device).synchronize()
        return self._read_out()

    def _solve_fn(self, contact, feet, stance, xref=None):
        """The bound mpcqp_solve launcher for these input buffers (stance range set)."""
        e = self._engine
        dv = self._dev
        # the exact stance count of this table: only the capacity class it needs launches
        e.set_stance_range(stance, stance)
        xr = dv["xref"] if xref is None else xref
        key = (contact.data_ptr(), feet.data_ptr(), xr.data_ptr())
        fn = self._solve_fns.get(key)
        if fn is None:
            if len(self._solve_fns) > 8:   # host-array xrefs (direct _solve_mpc calls) allocate fresh buffers
                self._solve_fns.clear()
            fn = self._solve_fns[key] = e.bind_solve(1, dv["x0"], xr, contact, feet, dv["robot"], dv["u0"],
                                                     dv["U"], dv["status"], dv["iters"])
        return fn

    def _mpc_tick(self, up):
        """An MPC tick after the upload: plan (integrate + reference trajectory) and the
        solve on the bound launchers, one readback and one synchronisation.  (A HIP graph
        of the three measured no faster on the GPU pool)"""
        from mpcqp._lib import PLAN_REFERENCE
        self._plan(PLAN_REFERENCE, up)
        return self._solve_dev(up["contact"], up["feet"], up["stance"])

    def _read_out(self):
        out = self._out_pinned.numpy()
        N12 = 12 * self.horizon
        U = out[:N12].astype(np.float64)
        status = int(out[N12:N12 + 1].view(np.int32)[0])
        if status in (3, 4, 5):   # TOO_LARGE / NONFINITE / UNSUPPORTED: no iterate, U = 0
            raise RuntimeError(f"mpcqp: robot solve failed with status {status}")
        if status != 0:
            # mpc.py:284-286 never checks is_success; the best iterate is returned, loudly
            warnings.warn(f"mpcqp: robot solve status {status}; returning the best iterate")
        return U
