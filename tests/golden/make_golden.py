"""Generate the golden fixtures in tests/golden/ FROM THE REFERENCE ITSELF.

Runs only in the build container (it reads /root/reference, which never
travels to the GPU box).  The reference's formulation functions are imported
with the four unavailable third-party modules stubbed (numba, pydrake,
qpsolvers, pinocchio -- none of them is called on the formulation path;
SURVEY.md Appendix A), then:

  formulation_N{N}.npz  inputs + the reference's own (H, g) for every case,
                        (C, lb, ub) for the first cases, and u* = the exact
                        optimum of the reference-built QP (oracle/qp.py dual
                        active set, float64) with its KKT residuals.
  gait_N{N}.npz         Gait.get_gait_table() (linear_mpc/gait.py:81-100) for
                        every gait member and iterations 0..2*period
  reftraj.npz           generate_reference_trajectory() (mpc.py:110-170) and
                        the update_mpc_if_needed pose integration (mpc.py:83-92)
  planner.npz           a 45-iteration control sequence through the reference's own
                        update_robot_state + update_mpc_if_needed (mpc.py:55-108, with
                        _solve_mpc replaced by a recorder), quat2ZYXangle / quat2matrix
                        (kinematics.py:40-71) on float32 quaternions, and
                        LegController.update's stance branch (leg_controller.py:86-89)

  formulation_full_N{N}.npz  the same for full (non-diagonal) Q and R (--full N): leg-block R
                        at N = 10 / 16, an R coupling every pair of legs at N = 20 / 24 (the
                        interior-point class's 12 x 12 stage weights), standing robots included

Usage:  python tests/golden/make_golden.py            (all horizons, subprocesses)
        python tests/golden/make_golden.py --horizon 10
        python tests/golden/make_golden.py --planner       (planner.npz only)
"""
import argparse
import os
import subprocess
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
HORIZONS = (10, 16, 20, 24, 32)


def stub_reference(horizon):
    sys.path[:0] = [f"{REF}/linear_mpc", f"{REF}/config", f"{REF}/utils"]
    nb = types.ModuleType("numba")
    nb.jit = lambda *a, **k: (lambda f: f)
    nb.vectorize = nb.jit
    nb.float32 = np.float32
    pda = types.ModuleType("pydrake.all")
    pda.MathematicalProgram = pda.Solve = pda.PiecewisePolynomial = None
    pd = types.ModuleType("pydrake")
    pd.all = pda
    qs = types.ModuleType("qpsolvers")
    qs.solve_qp = None
    sys.modules.update({"numba": nb, "pydrake": pd, "pydrake.all": pda, "qpsolvers": qs,
                        "pinocchio": types.ModuleType("pinocchio")})
    import linear_mpc_configs
    # Gait captures the horizon when the Enum is created (gait.py:47-50): set it first
    linear_mpc_configs.LinearMpcConfig.horizon = horizon
    import gait
    import mpc
    import robot_configs
    return linear_mpc_configs.LinearMpcConfig, robot_configs, mpc, gait


def gen(horizon):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "pympc-quadruped_amd")]
    LinearMpcConfig, robot_configs, mpc, gait = stub_reference(horizon)
    from oracle import qp as Q
    from mpcqp.synthetic import make_batch
    from mpcqp.params import robot_from_config

    N = horizon
    cfgs = {"a1": robot_configs.A1Config, "aliengo": robot_configs.AliengoConfig}
    gaits = ("trot10", "pace10", "bound8", "standing")
    names = ("a1", "aliengo")
    B = 16
    bt = make_batch(B, N, seed=4242 + N, gaits=gaits, robots=names)
    if N > 20:
        # the horizons only the interior-point class takes (N > kDenseN): beside the gait mix
        # (standing robots included) a sparse schedule (n well below 128) and a flight one (n = 0)
        rng = np.random.default_rng(777 + N)
        bt["contact"][1] = (rng.random((N, 4)) < 0.2).astype(np.float32)
        bt["contact"][2] = 0.0
    # per-robot records straight from the reference config classes
    robot_name = []
    for b in range(B):
        nm = "a1" if abs(bt["robot"][b][0] - 4.713) < 1e-3 else "aliengo"
        robot_name.append(nm)
        bt["robot"][b] = robot_from_config(cfgs[nm])
    Hs, gs, us, kkts, iters, rounding = [], [], [], [], [], []
    C0 = lb0 = ub0 = None
    Cs, lbs, ubs = [], [], []
    for b in range(B):
        c = mpc.ModelPredictiveController(LinearMpcConfig, cfgs[robot_name[b]])
        x0 = bt["x0"][b].copy()
        c.current_state = x0
        c.yaw = float(x0[2])
        c.pos_base_feet = [bt["feet"][b][i].astype(np.float64) for i in range(4)]
        Ac, Bc = c._generate_state_space_model()
        c._discretize_continuous_model(Ac, Bc)
        Ad, Bd = c._discretize_continuous_model(Ac, Bc)
        H, g = c._generate_QP_cost(Ad, Bd, c.current_state, bt["xref"][b].reshape(-1))
        C, lb, ub = c._generate_QP_constraints(bt["contact"][b].reshape(-1))
        x, y, info = Q.solve_qp_dual_active_set(H, g, C, lb, ub)
        k = Q.kkt_residuals(H, g, C, lb, ub, x, y)
        Hs.append(H)
        gs.append(g)
        us.append(x)
        kkts.append([k["stationarity"], k["primal"], k["dual"], k["complementarity"]])
        iters.append(info["iterations"])
        if b < (2 if N <= 20 else 1):
            Cs.append(C); lbs.append(lb); ubs.append(ub)
        # u* is certified: the fixture is only as good as its optimum
        assert max(kkts[-1]) < 1e-7, (N, b, kkts[-1])
        rounding.append(len(info.get("rounding_accept", [])))
    # full H only for the first cases (size); every case keeps H @ probe vectors,
    # a size-independent pin of the whole matrix
    nH = 2 if N <= 16 else 1 if N <= 20 else 0
    probe = np.random.default_rng(99).standard_normal((2, 12 * N))
    probe[0] = 1.0
    Hprobe = np.array([[H @ v for v in probe] for H in Hs])
    out = dict(x0=bt["x0"], xref=bt["xref"], contact=bt["contact"], feet=bt["feet"], robot=bt["robot"],
               robot_name=np.array(robot_name), H=np.array(Hs[:nH]), H_probe=Hprobe, probe=probe,
               g=np.array(gs), u_star=np.array(us),
               kkt=np.array(kkts), iterations=np.array(iters), rounding_stops=np.array(rounding),
               C=np.array(Cs), lb=np.array(lbs),
               ub=np.array(ubs), horizon=N, dt=0.05)
    np.savez_compressed(os.path.join(HERE, f"formulation_N{N}.npz"), **out)

    # gait tables (linear_mpc/gait.py:16-22, :76-100)
    tables = {}
    for member in gait.Gait:
        rows = []
        for it in range(0, 2 * member.num_segment * 20 + 1, 20):
            member.set_iteration(20, it)
            rows.append(member.get_gait_table().copy())
        tables[member._name_] = np.array(rows)   # Enum key (Gait.name is overridden, gait.py:52-54)
    np.savez_compressed(os.path.join(HERE, f"gait_N{N}.npz"), **tables)

    if N == 16:
        gen_reftraj(LinearMpcConfig, robot_configs, mpc)
    print(f"N={N}: max KKT {np.array(kkts).max():.2e}, iterations {iters}, rounding-level stops {rounding}")


def full_weights(seed, cross_leg=False):
    """A symmetric positive-semidefinite Q coupling the moving state components (the
    reference's diagonal scaled by a correlation matrix, |rho| <= 0.4; state 12 keeps
    weight 0) and an R with full 3 x 3 leg blocks (mpc.py:49-52 take whole matrices) --
    or, cross_leg, an R coupling every pair of legs (the diagonal scaled by a dense random
    correlation matrix)."""
    rng = np.random.default_rng(seed)
    C = np.eye(13)
    for _ in range(12):
        i, j = rng.choice(12, size=2, replace=False)
        C[i, j] = C[j, i] = rng.uniform(-0.4, 0.4)
    w, V = np.linalg.eigh(C)
    C = V @ np.diag(np.maximum(w, 0.05)) @ V.T
    d = np.sqrt(np.diag(C))
    C = C / np.outer(d, d)
    sq = np.sqrt(np.array([5., 5., 10., 10., 10., 50., 0.01, 0.01, 0.2, 0.2, 0.2, 0.2, 0.]))
    Q = np.outer(sq, sq) * C
    R = np.diag([1e-5] * 12)
    for leg in range(4):
        S = rng.uniform(-0.3, 0.3, size=(3, 3))
        R[3 * leg:3 * leg + 3, 3 * leg:3 * leg + 3] += 1e-5 * (S @ S.T)
    if cross_leg:
        A = rng.standard_normal((12, 12))
        Cr = A @ A.T / 12.0 + 0.5 * np.eye(12)
        dr = np.sqrt(np.diag(Cr))
        R = 1e-5 * Cr / np.outer(dr, dr)
    return 0.5 * (Q + Q.T), 0.5 * (R + R.T)


def gen_full(horizon):
    """formulation_full_N{N}.npz: the reference's own H, g for full (non-diagonal) Q and R
    (a LinearMpcConfig subclass carrying them, mpc.py:49-52), and the exact optimum u* of
    that QP -- pins the oracle's and the engine's general-weight path."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "pympc-quadruped_amd")]
    LinearMpcConfig, robot_configs, mpc, gait = stub_reference(horizon)
    from oracle import qp as Q
    from mpcqp.synthetic import make_batch
    from mpcqp.params import robot_from_config
    N = horizon
    Qf, Rf = full_weights(500 + N, cross_leg=N >= 20)

    class FullWeights(LinearMpcConfig):
        Q = Qf
        R = Rf

    cfgs = {"a1": robot_configs.A1Config, "aliengo": robot_configs.AliengoConfig}
    B = 8
    bt = make_batch(B, N, seed=5151 + N, gaits=("trot10", "pace10", "bound8", "standing"), robots=("a1", "aliengo"))
    names, Hp, gs, us = [], [], [], []
    probe = np.random.default_rng(98).standard_normal((2, 12 * N))
    for b in range(B):
        nm = "a1" if abs(bt["robot"][b][0] - 4.713) < 1e-3 else "aliengo"
        names.append(nm)
        bt["robot"][b] = robot_from_config(cfgs[nm])
        c = mpc.ModelPredictiveController(FullWeights, cfgs[nm])
        x0 = bt["x0"][b].copy()
        c.current_state = x0
        c.yaw = float(x0[2])
        c.pos_base_feet = [bt["feet"][b][i].astype(np.float64) for i in range(4)]
        Ac, Bc = c._generate_state_space_model()
        Ad, Bd = c._discretize_continuous_model(Ac, Bc)
        H, g = c._generate_QP_cost(Ad, Bd, c.current_state, bt["xref"][b].reshape(-1))
        C, lb, ub = c._generate_QP_constraints(bt["contact"][b].reshape(-1))
        x, y, info = Q.solve_qp_dual_active_set(H, g, C, lb, ub)
        k = Q.kkt_residuals(H, g, C, lb, ub, x, y)
        assert max(k["stationarity"], k["primal"], k["dual"], k["complementarity"]) < 1e-7, (N, b, k)
        Hp.append([H @ v for v in probe])
        gs.append(g)
        us.append(x)
    np.savez_compressed(os.path.join(HERE, f"formulation_full_N{N}.npz"), x0=bt["x0"], xref=bt["xref"],
                        contact=bt["contact"], feet=bt["feet"], robot=bt["robot"], robot_name=np.array(names),
                        Q=Qf, R=Rf, H_probe=np.array(Hp), probe=probe, g=np.array(gs), u_star=np.array(us),
                        horizon=N, dt=0.05)
    print(f"full weights N={N}: {B} cases, stance counts {[int(v) for v in (bt['contact'] > 0).reshape(B, -1).sum(1)]}")


class _FakeRobotData:
    def __init__(self, R):
        self.R_base = R


def gen_reftraj(LinearMpcConfig, robot_configs, mpc):
    """generate_reference_trajectory + update_mpc_if_needed integrators (mpc.py:81-170)."""
    rng = np.random.default_rng(77)
    cases = []
    for k in range(12):
        c = mpc.ModelPredictiveController(LinearMpcConfig, robot_configs.AliengoConfig)
        x0 = np.zeros(13, dtype=np.float32)
        x0[:3] = rng.uniform(-0.1, 0.1, 3)
        x0[2] = rng.uniform(-3, 3)
        x0[3:6] = [rng.uniform(-1, 1), rng.uniform(-1, 1), 0.38]
        x0[9:12] = [rng.uniform(-0.5, 1.5), rng.uniform(-0.3, 0.3), 0.0]
        x0[12] = -9.81
        c.current_state = x0
        c.yaw = float(x0[2])
        c.roll_init, c.pitch_init = 0.0, 0.0
        c.is_initialized = True
        yaw = float(x0[2])
        R = np.array([[np.cos(yaw), -np.sin(yaw), 0], [np.sin(yaw), np.cos(yaw), 0], [0, 0, 1]])
        c._ModelPredictiveController__robot_data = _FakeRobotData(R)
        v_body = np.array([rng.uniform(0, 1.5), 0.0, 0.0])
        yaw_rate = float(rng.uniform(-0.5, 0.5))
        # run the integrators for a few ticks (iteration_between_mpc = 20, so no solve
        # is triggered except at multiples of 20 -- we call the pieces directly)
        seq = []
        for tick in range(3):
            vel_des = c._ModelPredictiveController__robot_data.R_base @ v_body
            if c.is_first_run:
                c.xpos_base_desired, c.ypos_base_desired, c.yaw_desired = 0.0, 0.0, c.yaw
                c.is_first_run = False
            else:
                c.xpos_base_desired += c.dt_control * vel_des[0]
                c.ypos_base_desired += c.dt_control * vel_des[1]
                c.yaw_desired = c.yaw + c.dt_control * yaw_rate
            X = c.generate_reference_trajectory(vel_des, yaw_rate)
            seq.append(X.copy())
        cases.append(dict(x0=x0, v_body=v_body, yaw_rate=yaw_rate, R=R, X=np.array(seq),
                          roll_init=c.roll_init, pitch_init=c.pitch_init))
    np.savez_compressed(os.path.join(HERE, "reftraj.npz"),
                        x0=np.array([c_["x0"] for c_ in cases]),
                        v_body=np.array([c_["v_body"] for c_ in cases]),
                        yaw_rate=np.array([c_["yaw_rate"] for c_ in cases]),
                        R=np.array([c_["R"] for c_ in cases]),
                        X=np.array([c_["X"] for c_ in cases]),
                        roll_init=np.array([c_["roll_init"] for c_ in cases]),
                        pitch_init=np.array([c_["pitch_init"] for c_ in cases]))


class _PlanRobotData:
    """The RobotData attributes update_robot_state / update_mpc_if_needed /
    LegController.update read (robot_data.py:59-190), set directly."""


def gen_planner():
    """planner.npz: the reference's own per-iteration planner outputs."""
    import contextlib
    import io
    sys.path[:0] = [ROOT]
    LinearMpcConfig, robot_configs, mpc, gait = stub_reference(16)
    import kinematics
    import leg_controller
    rng = np.random.default_rng(2024)
    B, T = 8, 45
    members = [gait.Gait.TROTTING10, gait.Gait.PACING16, gait.Gait.STANDING, gait.Gait.TROTTING16,
               gait.Gait.JUMPING16, gait.Gait.PACING10, gait.Gait.TROTTING10, gait.Gait.STANDING]
    quat = np.zeros((B, T, 4), np.float32)
    pos = np.zeros((B, T, 3), np.float32)
    omega = np.zeros((B, T, 3), np.float32)
    vel = np.zeros((B, T, 3), np.float32)
    v_body = np.zeros((B, 3))
    yaw_rate = np.zeros(B)
    x0 = np.zeros((B, T, 13), np.float32)
    rot = np.zeros((B, T, 3, 3), np.float32)
    rpy = np.zeros((B, T, 3))
    xref = np.zeros((B, 3, 16 * 13), np.float32)
    table = np.zeros((B, 3, 16 * 4), np.float32)
    pstate = np.zeros((B, 3, 5))
    for b in range(B):
        c = mpc.ModelPredictiveController(LinearMpcConfig, robot_configs.AliengoConfig)
        v_body[b] = [rng.uniform(-0.5, 1.5), rng.uniform(-0.4, 0.4), 0.0]
        yaw_rate[b] = rng.uniform(-0.8, 0.8)
        # a drifting base pose: roll/pitch wobble, a yaw that sweeps past +-pi for some robots
        rpy0 = np.array([rng.uniform(-0.15, 0.15), rng.uniform(-0.15, 0.15), rng.uniform(-3.1, 3.1)])
        p0 = np.array([rng.uniform(-1, 1), rng.uniform(-1, 1), 0.38])
        k_mpc = 0
        for t in range(T):
            r, p, y = rpy0 + np.array([0.05 * np.sin(0.3 * t), 0.04 * np.cos(0.2 * t), 0.02 * t])
            cr, sr, cp, sp, cy, sy = np.cos(r / 2), np.sin(r / 2), np.cos(p / 2), np.sin(p / 2), \
                np.cos(y / 2), np.sin(y / 2)
            q = np.array([cr * cp * cy + sr * sp * sy, sr * cp * cy - cr * sp * sy,
                          cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy], dtype=np.float32)
            quat[b, t] = q
            # positions drift off the desired track so the +-0.1 clamp engages (mpc.py:129-137)
            pos[b, t] = p0 + np.array([0.004 * t * (1 + b % 3), -0.003 * t * (b % 2), 0.01 * np.sin(t)])
            omega[b, t] = rng.uniform(-0.5, 0.5, 3)
            vel[b, t] = [v_body[b][0] + rng.uniform(-0.3, 0.3), rng.uniform(-0.3, 0.3), rng.uniform(-.1, .1)]
            rd = _PlanRobotData()
            rd.quat_base = quat[b, t]
            rd.pos_base = pos[b, t]
            rd.ang_vel_base = omega[b, t]
            rd.lin_vel_base = vel[b, t]
            rd.R_base = kinematics.quat2matrix(quat[b, t])      # robot_data.py:75
            rd.pos_base_feet = [np.zeros(3)] * 4
            rot[b, t] = rd.R_base
            rpy[b, t] = kinematics.quat2ZYXangle(quat[b, t])
            members[b].set_iteration(c.iterations_between_mpc, t)
            gt = members[b].get_gait_table()
            rec = {}
            c._solve_mpc = lambda ref, g, solver='drake', debug=False, rec=rec: \
                (rec.update(ref=ref.copy(), g=np.array(g).copy()), np.zeros(12 * 16))[1]
            c.update_robot_state(rd)
            with contextlib.redirect_stdout(io.StringIO()):
                c.update_mpc_if_needed(t, v_body[b].tolist(), float(yaw_rate[b]), gt)
            x0[b, t] = c.current_state
            if t % c.iterations_between_mpc == 0:
                xref[b, k_mpc] = rec["ref"]
                table[b, k_mpc] = rec["g"]
                pstate[b, k_mpc] = [c.xpos_base_desired, c.ypos_base_desired, c.yaw_desired,
                                    float(c.roll_init), float(c.pitch_init)]
                k_mpc += 1
    # stance torques through LegController.update with every leg in stance
    lc = leg_controller.LegController(np.eye(3), np.eye(3))
    jv = rng.standard_normal((B, 4, 3, 18)).astype(np.float32)
    forces = rng.uniform(-40, 120, (B, 12)).astype(np.float32)
    tau = np.zeros((B, 12), np.float32)
    for b in range(B):
        rd = _PlanRobotData()
        rd.Jv_feet = [jv[b, leg] for leg in range(4)]
        rd.R_base = np.eye(3)
        rd.base_vel_base_feet = np.zeros((4, 3))
        rd.base_pos_base_feet = np.zeros((4, 3))
        tau[b] = lc.update(rd, forces[b], [0, 0, 0, 0], np.zeros((4, 3)), np.zeros((4, 3)))
    gait_rec = np.array([[m.num_segment, *m.stance_offsets, *m.stance_durations] for m in members], np.int32)
    np.savez_compressed(os.path.join(HERE, "planner.npz"), quat=quat, pos=pos, omega=omega, vel=vel,
                        v_body=v_body, yaw_rate=yaw_rate, x0=x0, rot=rot, rpy=rpy, xref=xref, table=table,
                        plan_state=pstate, gait=gait_rec, jv=jv, forces=forces, tau=tau, horizon=16,
                        iterations_between_mpc=20, height=0.38)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--horizon", type=int, default=0)
    ap.add_argument("--planner", action="store_true")
    ap.add_argument("--full", type=int, default=0, help="formulation_full_N{N}.npz only")
    a = ap.parse_args()
    if a.full:
        gen_full(a.full)
    elif a.planner:
        gen_planner()
    elif a.horizon:
        gen(a.horizon)
    else:
        for n in HORIZONS:
            subprocess.run([sys.executable, __file__, "--horizon", str(n)], check=True)
