"""Batched control tick on the device: the loop body the reference runs per robot.

``BatchedController`` is B copies of the reference's per-robot objects -- one
``Gait``, one ``ModelPredictiveController`` and the stance branch of one
``LegController`` -- advanced together, so a whole fleet's control iteration is
three HIP launches with every intermediate resident in HBM:

  mpcqp_plan            Gait.set_iteration / get_gait_table          gait.py:76-100
                        ModelPredictiveController.update_robot_state mpc.py:55-79
                        update_mpc_if_needed integrators, X_ref      mpc.py:81-170
  mpcqp_solve           _solve_mpc on MPC ticks                      mpc.py:262-290
  mpcqp_stance_torques  LegController stance branch                  leg_controller.py:86-89

The per-robot Python loop it replaces is scripts/isaacgym_a1.py:117-151 (which
copies every robot's root state to the host, ``.cpu().numpy()``); ``tick`` takes
the simulator's root-state tensor as it lies on the device.
"""
import numpy as np
import torch

from ._lib import PLAN_REFERENCE, PLAN_STRIDE
from .engine import LinearMpc
from .params import DT_MPC, Q_DIAG, R_DIAG, ROBOT_PRESETS, gait_record


class BatchedController:
    """Args:
      batch:    number of robots B
      horizon:  MPC horizon N (linear_mpc_configs.py:11)
      robot:    preset name / RobotConfig class / packed record, or [B,16] records
      gait:     one gait (GAITS key, Gait member name, or (period, offsets, durations))
                or a list of B of them
      iterations_between_mpc: linear_mpc_configs.py:7 (20)
      dt_control: linear_mpc_configs.py:6 (0.001)
      height:   desired CoM height(s) (robot_configs.py:23,42); default from the preset
      warm_start: remember each robot's active set between MPC ticks (LinearMpc.set_warm_start)
    """

    def __init__(self, batch, horizon=16, robot="aliengo", gait="trot10", iterations_between_mpc=20,
                 dt_control=0.001, gravity=9.81, height=None, dt=DT_MPC, Q=Q_DIAG, R=R_DIAG,
                 device="cuda:0", max_iter=0, max_stance=0, warm_start=True):
        self.B = int(batch)
        self.N = int(horizon)
        self.iterations_between_mpc = int(iterations_between_mpc)
        per_robot = not isinstance(robot, str) and np.ndim(robot) == 2
        self.engine = LinearMpc(horizon=self.N, robot=None if per_robot else robot, dt=dt, Q=Q, R=R,
                                device=device, max_iter=max_iter, max_stance=max_stance)
        self.engine.set_planner(dt_control=dt_control, gravity=gravity)
        if warm_start:   # the fleet is solved tick after tick: remember each robot's active set
            self.engine.set_warm_start(int(batch))
        dev = self.engine.device
        self.device = dev
        B, N = self.B, self.N
        if per_robot:
            self.robot = torch.as_tensor(np.asarray(robot, dtype=np.float32)).to(dev).contiguous()
        else:
            rec = self.engine.default_robot
            self.robot = torch.as_tensor(np.tile(rec, (B, 1))).to(dev).contiguous()
        single = isinstance(gait, str) or (isinstance(gait, (tuple, list)) and len(gait) == 3
                                           and np.isscalar(gait[0]) and not isinstance(gait[0], str))
        gaits = [gait] * B if single else list(gait)
        if len(gaits) != B:
            raise ValueError(f"expected one gait or {B} of them, got {len(gaits)}")
        g = np.stack([gait_record(x) for x in gaits])
        self.gait = torch.as_tensor(g).to(dev).contiguous()
        self._period = self.gait[:, 0].clone()
        if height is None:
            if isinstance(robot, str):
                height = ROBOT_PRESETS[robot].get("height", 0.38)
            elif hasattr(robot, "base_height_des"):
                height = robot.base_height_des
            else:
                raise ValueError("height is required for a packed robot record")
        self.height = torch.as_tensor(np.broadcast_to(np.asarray(height, dtype=np.float32), (B,)).copy()).to(dev)
        f32 = dict(dtype=torch.float32, device=dev)
        self.plan_state = torch.zeros((B, PLAN_STRIDE), dtype=torch.float64, device=dev)
        self.x0 = torch.zeros((B, 13), **f32)
        self.xref = torch.zeros((B, N, 13), **f32)
        self.contact = torch.zeros((B, N, 4), **f32)
        self.u0 = torch.zeros((B, 12), **f32)
        self.tau = torch.zeros((B, 12), **f32)
        self.status = torch.zeros((B,), dtype=torch.int32, device=dev)
        self.iterations = torch.zeros((B,), dtype=torch.int32, device=dev)
        self.iteration = torch.zeros((B,), dtype=torch.int32, device=dev)

    def reset(self, robots=None):
        """First-run semantics again (mpc.py:56-60,84-87) for all or some robots."""
        if robots is None:
            self.plan_state.zero_()
        else:
            self.plan_state[robots] = 0.0

    def _cmd(self, v, shape):
        t = torch.as_tensor(v, dtype=torch.float64)
        return t.to(self.device).expand(shape).contiguous()

    def tick(self, iter_counter, vel_body_des, yaw_rate_des, feet, root_states=None, quat=None, pos=None,
             omega=None, vel=None, rot=None):
        """One control iteration for every robot; returns u0 [B,12] (device).

        The contact forces are re-solved when ``iter_counter % iterations_between_mpc
        == 0`` and held otherwise (mpc.py:95-106).  feet [B,4,3] are the foot positions
        relative to the CoM in the world frame (robot_data.pos_base_feet)."""
        B = self.B
        ibm = self.iterations_between_mpc
        mpc_tick = iter_counter % ibm == 0
        flags = PLAN_REFERENCE if mpc_tick else 0
        if mpc_tick:
            # gait.py:76-78: iteration = floor(iter / iterations_between_mpc) % period
            torch.remainder(torch.full_like(self._period, iter_counter // ibm), self._period, out=self.iteration)
        vb = self._cmd(vel_body_des, (B, 3))
        yr = self._cmd(yaw_rate_des, (B,))
        if root_states is not None:
            rs = root_states if root_states.dtype == torch.float32 and root_states.is_contiguous() \
                else root_states.to(torch.float32).contiguous()
            self.engine.plan(flags, self.plan_state, self.x0, vb, yr, root_states=rs, gait=self.gait,
                             iteration=self.iteration, height_des=self.height, xref=self.xref,
                             contact=self.contact)
        else:
            c = [t.to(self.device, torch.float32).contiguous() for t in (quat, pos, omega, vel)]
            r = rot.to(self.device, torch.float32).contiguous() if rot is not None else None
            self.engine.plan(flags, self.plan_state, self.x0, vb, yr, quat=c[0], pos=c[1], omega=c[2],
                             vel=c[3], rot=r, gait=self.gait, iteration=self.iteration,
                             height_des=self.height, xref=self.xref, contact=self.contact)
        if mpc_tick:
            ft = feet.to(self.device, torch.float32).contiguous()
            self.engine.solve_raw(B, self.x0, self.xref, self.contact, ft, self.robot, self.u0,
                                  status=self.status, iters=self.iterations)
        return self.u0

    def torques(self, jac, stance):
        """Stance-leg joint torques into self.tau (leg_controller.py:86-89).

        jac [B,4,3,3]: each leg's 3x3 block of its foot Jacobian; stance [B,4] > 0 for
        legs whose swing state is 0 (leg_controller.py:77).  Swing-leg entries of tau
        keep whatever the swing controller wrote."""
        j = jac.to(self.device, torch.float32).contiguous()
        s = stance.to(self.device, torch.float32).contiguous()
        self.engine.stance_torques(j, s, self.u0, self.tau, stance_stride=s.shape[-1])
        return self.tau
