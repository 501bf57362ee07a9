"""GPU parity of the hot path's callers: mpcqp_plan,
mpcqp_plan_root_states and mpcqp_stance_torques against the reference's own
recorded outputs (tests/golden/planner.npz, gait_N*.npz) and the CPU oracle
(oracle/planner.py), through the C ABI (-m gpu).

Tolerances: x0 / R_base to 1 float32 ulp (the reference squares quaternion
components with NumPy's SIMD power routine, the device and the oracle multiply);
X_ref to 1e-6 absolute (NumPy 2.2 fixture vs the pinned 1.24 promotion, see
tests/test_oracle.py); gait tables bit-exact; the planner state to 3e-7 (a float32 ulp: the NumPy 2.2 fixture rounds the clamp)."""
import os

import numpy as np
import pytest

from helpers import oracle_solution, rel_err_u0

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
TOL_U0 = 1e-4


def _load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def _engine(N, **kw):
    from mpcqp import LinearMpc
    return LinearMpc(horizon=N, robot="aliengo", **kw)


def _dev(a, dtype=None):
    import torch
    t = torch.as_tensor(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.to("cuda:0").contiguous()


class _Plan:
    """Device buffers for B robots of one engine."""

    def __init__(self, eng, B, N, gait=None, height=0.38):
        import torch
        self.eng, self.B, self.N = eng, B, N
        f32 = dict(dtype=torch.float32, device="cuda:0")
        self.state = torch.zeros((B, 8), dtype=torch.float64, device="cuda:0")
        self.x0 = torch.zeros((B, 13), **f32)
        self.xref = torch.zeros((B, N, 13), **f32)
        self.contact = torch.full((B, N, 4), -1.0, **f32)
        self.height = torch.full((B,), height, **f32)
        self.gait = _dev(gait) if gait is not None else None
        self.iteration = torch.zeros((B,), dtype=torch.int32, device="cuda:0")

    def run(self, flags, vb, yr, iteration=None, **inputs):
        import torch
        if iteration is not None:
            self.iteration.copy_(torch.as_tensor(np.asarray(iteration, dtype=np.int32)))
        self.eng.plan(flags, self.state, self.x0, _dev(vb, torch.float64), _dev(yr, torch.float64),
                      gait=self.gait, iteration=self.iteration if self.gait is not None else None,
                      height_des=self.height, xref=self.xref,
                      contact=self.contact if self.gait is not None else None, **inputs)
        torch.cuda.synchronize()


def _sequence(z, root_layout):
    """Run planner.npz's control sequence on the device; returns per-tick x0 and the
    MPC-tick xref / contact / state."""
    from mpcqp._lib import PLAN_REFERENCE
    B, T = z["quat"].shape[:2]
    N, ibm = int(z["horizon"]), int(z["iterations_between_mpc"])
    p = _Plan(_engine(N), B, N, gait=z["gait"], height=float(z["height"]))
    xs, xr, ct, st = [], [], [], []
    for t in range(T):
        tick = t % ibm == 0
        it = (t // ibm) % z["gait"][:, 0]
        if root_layout:
            q = z["quat"][:, t]
            rs = np.concatenate([z["pos"][:, t], q[:, 1:4], q[:, 0:1], z["vel"][:, t], z["omega"][:, t]], 1)
            p.run(PLAN_REFERENCE if tick else 0, z["v_body"], z["yaw_rate"], it, root_states=_dev(rs))
        else:
            p.run(PLAN_REFERENCE if tick else 0, z["v_body"], z["yaw_rate"], it, quat=_dev(z["quat"][:, t]),
                  pos=_dev(z["pos"][:, t]), omega=_dev(z["omega"][:, t]), vel=_dev(z["vel"][:, t]))
        xs.append(p.x0.cpu().numpy())
        if tick:
            xr.append(p.xref.cpu().numpy().reshape(B, -1))
            ct.append(p.contact.cpu().numpy().reshape(B, -1))
            st.append(p.state.cpu().numpy()[:, :5])
    return (np.stack(xs, 1), np.stack(xr, 1), np.stack(ct, 1), np.stack(st, 1))


@pytest.mark.parametrize("root_layout", [False, True])
def test_plan_matches_reference_sequence(root_layout):
    """45 control iterations (3 MPC ticks) vs the reference's recorded planner outputs."""
    z = _load("planner.npz")
    xs, xr, ct, st = _sequence(z, root_layout)
    np.testing.assert_allclose(xs, z["x0"], rtol=2.4e-7, atol=0)
    np.testing.assert_allclose(xr, z["xref"], rtol=0, atol=1e-6)
    np.testing.assert_array_equal(ct, z["table"])
    # the fixture's clamp ``current_state[3] + 0.1`` is float32 under NumPy 2.2 (NEP 50)
    np.testing.assert_allclose(st, z["plan_state"], rtol=0, atol=3e-7)


def test_root_state_layout_is_the_same_computation():
    z = _load("planner.npz")
    a = _sequence(z, False)
    b = _sequence(z, True)
    for u, v in zip(a, b):
        np.testing.assert_array_equal(u, v)


@pytest.mark.parametrize("N", [10, 16, 20])
def test_gait_tables_match_reference(N):
    """Gait.get_gait_table for every member at iterations 0..2*period (gait.py:76-100)."""
    from mpcqp._lib import PLAN_REFERENCE
    from mpcqp.params import GAIT_MEMBERS, gait_record
    z = _load(f"gait_N{N}.npz")
    names = [k for k in z.files]
    recs = np.stack([gait_record(GAIT_MEMBERS[k]) for k in names])
    steps = max(z[k].shape[0] for k in names)
    B = len(names)
    p = _Plan(_engine(N), B, N, gait=recs)
    ident = dict(quat=_dev(np.tile([1, 0, 0, 0], (B, 1)).astype(np.float32)), pos=_dev(np.zeros((B, 3), np.float32)),
                 omega=_dev(np.zeros((B, 3), np.float32)), vel=_dev(np.zeros((B, 3), np.float32)))
    for k in range(steps):
        it = np.array([(k % recs[i, 0]) if k < z[names[i]].shape[0] else 0 for i in range(B)])
        p.run(PLAN_REFERENCE, np.zeros((B, 3)), np.zeros(B), it, **ident)
        c = p.contact.cpu().numpy().reshape(B, -1)
        for i, nm in enumerate(names):
            if k < z[nm].shape[0]:
                np.testing.assert_array_equal(c[i], z[nm][k], err_msg=f"{nm} k={k}")


def test_plan_large_batch_matches_oracle():
    """B = 3000 robots (ragged last workgroup), mixed gaits, 41 iterations incl. 3 MPC
    ticks, per-robot commands, vs oracle/planner.py robot by robot."""
    from mpcqp._lib import PLAN_REFERENCE
    from mpcqp.params import GAITS, gait_record
    from oracle.planner import PlannerOracle, gait_table, quat2matrix, world_velocity
    rng = np.random.default_rng(7)
    B, N, T, ibm = 3000, 16, 41, 20
    names = ["trot10", "pace16", "bound8", "standing", "jump16", "trot16", "pace10"]
    gsel = rng.integers(0, len(names), B)
    recs = np.stack([gait_record(names[i]) for i in gsel])
    q = rng.standard_normal((B, 4))
    q[:, 0] = np.abs(q[:, 0]) + 2.0
    q = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)
    vb = np.stack([rng.uniform(-1, 2, B), rng.uniform(-0.5, 0.5, B), np.zeros(B)], 1)
    yr = rng.uniform(-1, 1, B)
    pos0 = rng.uniform(-2, 2, (B, 3)).astype(np.float32)
    p = _Plan(_engine(N), B, N, gait=recs)
    check = rng.choice(B, 96, replace=False)
    check[0], check[1] = 0, B - 1
    oracles = {b: PlannerOracle(N, 0.38) for b in check}
    for t in range(T):
        pos = (pos0 + 0.01 * t * rng.uniform(-1, 1, (B, 3))).astype(np.float32)
        omega = rng.uniform(-1, 1, (B, 3)).astype(np.float32)
        vel = (vb + rng.uniform(-0.4, 0.4, (B, 3))).astype(np.float32)
        tick = t % ibm == 0
        it = (t // ibm) % recs[:, 0]
        p.run(PLAN_REFERENCE if tick else 0, vb, yr, it, quat=_dev(q), pos=_dev(pos), omega=_dev(omega),
              vel=_dev(vel))
        x0 = p.x0.cpu().numpy()
        xr = p.xref.cpu().numpy()
        ct = p.contact.cpu().numpy()
        st = p.state.cpu().numpy()
        for b in check:
            o = oracles[b]
            xs = o.update_robot_state(q[b], pos[b], omega[b], vel[b])
            np.testing.assert_allclose(x0[b], xs, rtol=2.4e-7, atol=0)
            v = world_velocity(quat2matrix(q[b]), vb[b])
            o.integrate(v, yr[b])
            if tick:
                X = o.reference_trajectory(v, yr[b])
                np.testing.assert_allclose(xr[b], X, rtol=0, atol=2e-6, err_msg=f"robot {b} t={t}")
                period, off, dur = GAITS[names[gsel[b]]]
                np.testing.assert_array_equal(ct[b], gait_table(period, off, dur, int(it[b]), N))
            np.testing.assert_allclose(st[b, :5], o.state_record()[:5], rtol=0, atol=1e-7)


def test_reference_only_flag_skips_integrators():
    """REFERENCE | NO_INTEGRATE == generate_reference_trajectory alone (mpc.py:110-170)."""
    import torch
    from mpcqp._lib import PLAN_NO_INTEGRATE, PLAN_REFERENCE
    from oracle.planner import PlannerOracle, quat2matrix, world_velocity
    B, N = 5, 10
    rng = np.random.default_rng(3)
    p = _Plan(_engine(N), B, N)
    q = np.tile(np.array([0.99, 0.05, -0.03, 0.1], np.float32), (B, 1))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    pos = rng.uniform(-1, 1, (B, 3)).astype(np.float32)
    vel = rng.uniform(-1, 1, (B, 3)).astype(np.float32)
    omega = np.zeros((B, 3), np.float32)
    vb, yr = rng.uniform(-1, 1, (B, 3)), rng.uniform(-1, 1, B)
    inp = dict(quat=_dev(q), pos=_dev(pos), omega=_dev(omega), vel=_dev(vel))
    os_ = [PlannerOracle(N, 0.38) for _ in range(B)]
    p.run(0, vb, yr, **inp)                                   # first integration
    for _ in range(2):
        p.run(PLAN_REFERENCE | PLAN_NO_INTEGRATE, vb, yr, **inp)
    xr = p.xref.cpu().numpy()
    for b in range(B):
        o = os_[b]
        o.update_robot_state(q[b], pos[b], omega[b], vel[b])
        v = world_velocity(quat2matrix(q[b]), vb[b])
        o.integrate(v, yr[b])
        o.reference_trajectory(v, yr[b])
        np.testing.assert_allclose(xr[b], o.reference_trajectory(v, yr[b]), rtol=0, atol=1e-6)
    assert torch.all(p.state[:, 5] == 1.0)


def test_stance_torques_match_reference_and_oracle():
    """tau = Jv^T (-f) (leg_controller.py:86-89): the reference's recorded torques, and
    the oracle on a large random batch; swing-leg entries are left untouched."""
    import torch
    from oracle.planner import stance_torques
    z = _load("planner.npz")
    eng = _engine(16)
    B = z["jv"].shape[0]
    jac = np.stack([[z["jv"][b, leg][:, 6 + 3 * leg:9 + 3 * leg] for leg in range(4)] for b in range(B)])
    tau = torch.zeros((B, 12), dtype=torch.float32, device="cuda:0")
    eng.stance_torques(_dev(jac), _dev(np.ones((B, 4), np.float32)), _dev(z["forces"]), tau)
    np.testing.assert_allclose(tau.cpu().numpy(), z["tau"], rtol=1e-6, atol=1e-4)

    rng = np.random.default_rng(11)
    B = 5000
    jac = rng.standard_normal((B, 4, 3, 3)).astype(np.float32)
    stance = (rng.random((B, 4)) < 0.6).astype(np.float32)
    u0 = rng.uniform(-50, 150, (B, 12)).astype(np.float32)
    tau = torch.full((B, 12), 7.0, dtype=torch.float32, device="cuda:0")
    eng.stance_torques(_dev(jac), _dev(stance), _dev(u0), tau)
    ref = stance_torques(jac, stance, u0, np.full((B, 12), 7.0, np.float32))
    np.testing.assert_allclose(tau.cpu().numpy(), ref, rtol=1e-5, atol=1e-3)
    assert np.all(tau.cpu().numpy()[np.repeat(stance == 0, 3, axis=1)] == 7.0)


def test_batched_controller_tick_matches_oracle_chain():
    """plan -> solve -> torques on the device == oracle planner -> oracle formulation +
    exact QP (GRF within 1e-4) over two MPC ticks, with the Isaac Gym root-state input."""
    import torch
    from mpcqp.controller import BatchedController
    from oracle.planner import PlannerOracle, gait_table, quat2matrix, world_velocity
    from oracle.planner import GAITS
    rng = np.random.default_rng(5)
    B, N, ibm = 24, 10, 20
    names = ["trot10", "pace10", "bound8"]
    gsel = [names[b % 3] for b in range(B)]
    ctl = BatchedController(B, horizon=N, robot="aliengo", gait=gsel, iterations_between_mpc=ibm)
    vb, yr = np.array([0.6, 0.0, 0.0]), 0.2
    feet = np.tile(np.array([[0.24, 0.13, -0.38], [0.24, -0.13, -0.38], [-0.24, 0.13, -0.38],
                             [-0.24, -0.13, -0.38]], np.float32), (B, 1, 1))
    feet += rng.uniform(-0.02, 0.02, feet.shape).astype(np.float32)
    oracles = [PlannerOracle(N, 0.38) for _ in range(B)]
    from mpcqp.params import ROBOT_PRESETS, pack_robot
    rec = pack_robot(ROBOT_PRESETS["aliengo"])
    for t in range(ibm + 1):
        q = np.tile(np.array([0.999, 0.01, -0.02, 0.03], np.float32), (B, 1))
        q += rng.uniform(-0.01, 0.01, q.shape).astype(np.float32)
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        pos = np.stack([0.6 * 0.001 * t + rng.uniform(-0.02, 0.02, B), rng.uniform(-0.02, 0.02, B),
                        0.38 + rng.uniform(-0.01, 0.01, B)], 1).astype(np.float32)
        vel = np.stack([0.6 + rng.uniform(-0.1, 0.1, B), rng.uniform(-0.05, 0.05, B), np.zeros(B)],
                       1).astype(np.float32)
        omega = rng.uniform(-0.1, 0.1, (B, 3)).astype(np.float32)
        rs = np.concatenate([pos, q[:, 1:4], q[:, 0:1], vel, omega], 1)
        u0 = ctl.tick(t, vb, yr, _dev(feet), root_states=_dev(rs)).cpu().numpy()
        status = ctl.status.cpu().numpy()
        for b in range(B):
            o = oracles[b]
            x0 = o.update_robot_state(q[b], pos[b], omega[b], vel[b])
            v = world_velocity(quat2matrix(q[b]), vb)
            o.integrate(v, yr)
            if t % ibm == 0:
                X = o.reference_trajectory(v, yr)
                period, off, dur = GAITS[gsel[b]]
                ct = gait_table(period, off, dur, (t // ibm) % period, N)
                bt = dict(x0=x0[None], xref=X[None], contact=ct[None], feet=feet[b:b + 1], robot=rec[None])
                x, _, _ = oracle_solution(bt, 0, N)
                assert status[b] == 0
                assert rel_err_u0(u0[b], x[:12]) < TOL_U0, (t, b, u0[b], x[:12])
    jac = rng.standard_normal((B, 4, 3, 3)).astype(np.float32)
    stance = np.ones((B, 4), np.float32)
    tau = ctl.torques(_dev(jac), _dev(stance)).cpu().numpy()
    ref = np.einsum("blrc,blr->blc", jac, -u0.reshape(B, 4, 3)).reshape(B, 12)
    np.testing.assert_allclose(tau, ref, rtol=1e-5, atol=1e-3)
    assert torch.isfinite(ctl.u0).all()
