"""GPU parity: the HIP engine vs the float64 oracle and the reference's own
fixtures, on identical inputs (-m gpu).  Every call goes through the C ABI
(libmpcqp.so via mpcqp.LinearMpc)."""
import os

import numpy as np
import pytest

from helpers import oracle_solution, rel_err_u0

TOL_U0 = 1e-4   # north_star: GRF within 1e-4 relative, norm-wise ||du0||_inf / ||u0*||_inf
# the precision the engine actually delivers (dense classes ~5e-7, the interior-point
# class ~2e-6 on these cases): a regression guard 10x tighter than the contract, so a
# build that loses digits (e.g. an explicit block-inverse sweep) fails here
TOL_ACHIEVED = 1e-5
# the interior-point class (n > 128) stops its active-set polish at a stationarity
# residual of 1e-10 x the gradient scale: on random contact patterns that leaves up to
# ~2e-5 (tools/parity_dist.py), still 5x inside the contract
TOL_ACHIEVED_IPM = 5e-5
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")

pytestmark = pytest.mark.gpu


def _engine(N, **kw):
    from mpcqp import LinearMpc
    return LinearMpc(horizon=N, robot="a1", **kw)


def _solve(eng, bt, **kw):
    res = eng.solve(bt["x0"], bt["xref"], bt["contact"], bt["feet"], robot=bt["robot"],
                    return_all=True, **kw)
    return (res.u0.cpu().numpy(), res.U.cpu().numpy().reshape(len(bt["x0"]), -1),
            res.status.cpu().numpy(), res.iterations.cpu().numpy())


@pytest.mark.parametrize("N,gaits,robots,tilt", [
    (10, ("trot10",), ("a1",), 0.0),
    (10, ("trot10", "pace10", "bound8"), ("a1", "aliengo"), 0.0),
    (10, ("trot10", "pace10", "bound8"), ("a1", "aliengo"), 15.0),
    (16, ("trot10", "pace10", "bound8"), ("a1",), 0.0),
    (20, ("trot10", "pace10", "bound8"), ("a1", "aliengo"), 15.0),
])
def test_u0_matches_oracle(N, gaits, robots, tilt):
    """N = 10 runs in the wave kernel (n = 60); N = 16/20 (n = 96/120) in the 8-wave class."""
    from mpcqp.synthetic import make_batch
    B = 24 if N == 10 else 12
    bt = make_batch(B, N, seed=11, gaits=gaits, robots=robots, tilt_deg=tilt)
    u0, U, status, _ = _solve(_engine(N), bt)
    assert (status == 0).all(), status
    worst = 0.0
    for b in range(B):
        x, _, _ = oracle_solution(bt, b, N)
        assert rel_err_u0(u0[b], x[:12]) < TOL_U0, (b, u0[b], x[:12])
        assert rel_err_u0(U[b], x) < TOL_U0, b
        worst = max(worst, rel_err_u0(u0[b], x[:12]), rel_err_u0(U[b], x))
    assert worst < TOL_ACHIEVED, worst


@pytest.mark.parametrize("N,B,gaits,robots,tilt,first", [
    (10, 1024, ("trot10",), ("a1",), 0.0, 0),                                    # config 2: held at once, no sort
    (10, 3000, ("trot10", "pace10", "bound8"), ("a1", "aliengo"), 0.0, 0),       # queued class 64, uneven XCD ranges
    (16, 700, ("trot10", "pace10", "bound8"), ("a1",), 0.0, 1),                  # class 96 taking the batch directly
    (20, 300, ("trot10", "pace10", "bound8"), ("a1", "aliengo"), 15.0, 2),       # class 128 directly
])
def test_dispatch_order_is_bitwise_neutral(N, B, gaits, robots, tilt, first):
    """mpcqp_set_order (ABI 6): dealing robots to workgroups by predicted cost changes only
    which workgroup solves a robot -- u0, U, status and iterations are bitwise those of the
    batch order, for class 64 (its XCD ranges sorted) and for classes 96 / 128 taking the
    batch directly (their segments sorted)."""
    from mpcqp.synthetic import make_batch
    bt = make_batch(B, N, seed=900 + N, gaits=gaits, robots=robots, tilt_deg=tilt)
    stance = (bt["contact"] > 0).reshape(B, -1).sum(1)
    out = []
    for mode in (0, 1):
        eng = _engine(N)
        if first:
            eng.set_stance_range(int(stance.min()), int(stance.max()))
        eng.set_order(mode)
        out.append(_solve(eng, bt))
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(a, b)
    assert (out[1][2] == 0).all()
    x, _, _ = oracle_solution(bt, B - 1, N)
    assert rel_err_u0(out[1][0][B - 1], x[:12]) < TOL_ACHIEVED


def test_dispatch_order_nonfinite_and_tied_keys():
    """The order kernel's key guards: non-finite states (key 0, dealt last; the robots
    report MPCQP_STATUS_NONFINITE) and a batch whose keys are all zero (v0 = vref_0: every
    robot in one bucket) keep the batch-order results bitwise."""
    from mpcqp.synthetic import make_batch
    N, B = 10, 3000
    bt = make_batch(B, N, seed=77, gaits=("trot10",), robots=("a1",))
    bt["x0"][7, 9] = np.nan
    bt["x0"][11, 10] = np.inf
    bt["x0"][13, 9] = 1e18   # finite, and its f32 key (1e36) too: the batch's largest key
    tied = {k: v.copy() for k, v in bt.items()}
    xr = tied["xref"].reshape(B, N, 13)
    tied["x0"][:, 9:11] = xr[:, 0, 9:11]
    for batch in (bt, tied):
        out = []
        for mode in (0, 1):
            eng = _engine(N)
            eng.set_order(mode)
            out.append(_solve(eng, batch))
        for a, b in zip(out[0], out[1]):
            assert np.array_equal(a, b)
    st = out[1][2]
    assert (st == 0).all()   # the tied batch
    st = _solve(_engine(N), bt)[2]
    assert st[7] == 4 and st[11] == 4, (st[7], st[11])
    # the huge but finite state is no NaN / inf row: it is solved (whatever its status), not
    # rejected, and every other robot -- all in the last key bucket behind it -- solves
    assert st[13] != 4, st[13]
    assert (np.delete(st, [7, 11, 13]) == 0).all()


def test_dispatch_order_batch_growth_and_graph_replay():
    """A class-64-only batch beyond four robots per CU takes a queue set for its dispatch order
    (include/mpcqp.h mpcqp_set_order: allocated on the first such call, and reallocated after a
    stream synchronisation when a later batch outgrows it).  A batch growing on one stream keeps
    the batch-order results bitwise, and a HIP graph captured after one call of the captured size
    (nothing left to allocate) replays to the eager results."""
    import torch
    from mpcqp.synthetic import make_batch
    N = 10
    full = make_batch(6000, N, seed=41, gaits=("trot10", "pace10"), robots=("a1",))
    eng, ref = _engine(N), _engine(N)
    ref.set_order(0)
    for B in (2000, 6000):   # 2000 > 1024 held at once: the first call allocates; 6000 grows the set
        bt = {k: v[:B] for k, v in full.items()}
        a, b = _solve(eng, bt), _solve(ref, bt)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    B = 6000
    dev = torch.device("cuda:0")
    d = {k: torch.as_tensor(full[k]).to(dev).float().contiguous() for k in ("x0", "xref", "contact", "feet", "robot")}
    u0 = torch.empty((B, 12), device=dev)
    st = torch.empty((B,), dtype=torch.int32, device=dev)
    it = torch.empty((B,), dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    args = (B, d["x0"], d["xref"], d["contact"], d["feet"], d["robot"], u0, None, st, it)
    eng.solve_raw(*args, stream=s)   # warm-up on the capture stream: its queue set exists
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        eng.solve_raw(*args, stream=s)
    u0.zero_()
    it.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(u0.cpu().numpy(), b[0])
    assert np.array_equal(it.cpu().numpy(), b[3])


def test_dispatch_order_batch_limits():
    """Class 64 sorts each XCD's range only up to kOrderMax = 8192 robots per range (a batch
    above 65 536 keeps the batch order) and never below kOrderMin = 64 or when the chip
    holds the batch at once: both sides of the upper limit, with the order on and off,
    give the same solutions."""
    from mpcqp.synthetic import make_batch
    N = 10
    full = make_batch(65544, N, seed=31, gaits=("trot10", "pace10"), robots=("a1",))
    for B in (65536, 65544):
        bt = {k: v[:B] for k, v in full.items()}
        out = []
        for mode in (0, 1):
            eng = _engine(N)
            eng.set_order(mode)
            out.append(_solve(eng, bt))
        for a, b in zip(out[0], out[1]):
            assert np.array_equal(a, b)
        assert (out[1][2] == 0).all()
        for b in (0, B // 3, B - 1):
            x, _, _ = oracle_solution(bt, b, N)
            assert rel_err_u0(out[1][0][b], x[:12]) < TOL_U0, (B, b)


@pytest.mark.parametrize("N", [10, 16, 20, 24, 32])
def test_reference_golden_fixtures(N):
    """u* of QPs built by the reference's own functions (tests/golden/make_golden.py):
    every case, standing schedules (n = 192 / 240, the interior-point class) included; at
    N = 24 / 32 (every robot in the interior-point class) also a sparse and a flight schedule,
    held to that class's precision guard."""
    z = np.load(os.path.join(GOLDEN, f"formulation_N{N}.npz"), allow_pickle=False)
    bt = {k: z[k] for k in ("x0", "xref", "contact", "feet", "robot")}
    u0, U, status, _ = _solve(_engine(N), bt)
    worst = 0.0
    for b in range(len(bt["x0"])):
        assert status[b] == 0, (b, status)
        assert rel_err_u0(u0[b], z["u_star"][b][:12]) < TOL_U0, (b, u0[b], z["u_star"][b][:12])
        assert rel_err_u0(U[b], z["u_star"][b]) < TOL_U0, b
        worst = max(worst, rel_err_u0(u0[b], z["u_star"][b][:12]), rel_err_u0(U[b], z["u_star"][b]))
    assert worst < (TOL_ACHIEVED if N <= 20 else TOL_ACHIEVED_IPM), worst
    if N > 20:
        assert np.all(U[2] == 0) and np.all(u0[2] == 0)   # the flight schedule


@pytest.mark.parametrize("N", [10, 16, 20, 24])
def test_reference_golden_full_weights(N):
    """u* of QPs the reference builds with full (non-diagonal) Q and R
    (formulation_full_N{N}.npz, mpc.py:49-52): the engine takes the same matrices
    (mpcqp_set_weights).  Leg-block R at N = 10 / 16, an R coupling every pair of legs at
    N = 20 / 24; N = 16 / 20 include standing robots (the interior-point class), N = 24 runs
    every robot there."""
    z = np.load(os.path.join(GOLDEN, f"formulation_full_N{N}.npz"), allow_pickle=False)
    bt = {k: z[k] for k in ("x0", "xref", "contact", "feet", "robot")}
    u0, U, status, _ = _solve(_engine(N, Q=z["Q"], R=z["R"]), bt)
    stance = (bt["contact"] > 0).reshape(len(bt["x0"]), -1).sum(1)
    worst, worst_ipm = 0.0, 0.0
    for b in range(len(bt["x0"])):
        assert status[b] == 0, (b, status)
        e = max(rel_err_u0(u0[b], z["u_star"][b][:12]), rel_err_u0(U[b], z["u_star"][b]))
        assert e < TOL_U0, (b, e)
        if 3 * stance[b] > 128 or N > 20:
            worst_ipm = max(worst_ipm, e)
        else:
            worst = max(worst, e)
    assert worst < TOL_ACHIEVED, worst
    assert worst_ipm < TOL_ACHIEVED_IPM, worst_ipm


def test_edge_cases():
    from mpcqp.synthetic import make_batch
    N = 10
    bt = make_batch(6, N, seed=5, gaits=("trot10",), robots=("a1",))
    bt["contact"][0] = 0.0                         # flight phase: every GRF is 0
    bt["xref"][1, 3, 4] = np.nan                   # non-finite input
    bt["contact"][2, :, :] = 1.0                   # standing: n = 120 -> the 8-wave class
    bt["contact"][3, 1:, :] = 0.0                  # single step of stance
    bt["contact"][3, 0, :] = 1.0
    u0, U, status, iters = _solve(_engine(N), bt)
    assert status[0] == 0 and np.all(u0[0] == 0) and np.all(U[0] == 0)
    assert status[1] == 4 and np.all(u0[1] == 0)
    assert status[2] == 0
    x, _, _ = oracle_solution(bt, 2, N)
    assert rel_err_u0(u0[2], x[:12]) < TOL_U0 and rel_err_u0(U[2], x) < TOL_U0
    assert status[3] == 0 and np.all(U[3][12:] == 0)
    x, _, _ = oracle_solution(bt, 3, N)
    assert rel_err_u0(u0[3], x[:12]) < TOL_U0
    for b in (4, 5):
        x, _, _ = oracle_solution(bt, b, N)
        assert status[b] == 0 and rel_err_u0(u0[b], x[:12]) < TOL_U0
    # standing at N = 20 (n = 240): the interior-point class, next to two class-128 robots
    bt20 = make_batch(3, 20, seed=6, gaits=("trot10",), robots=("a1",))
    bt20["contact"][1] = 1.0
    u20, U20, st20, _ = _solve(_engine(20), bt20)
    assert (st20 == 0).all(), st20
    for b in range(3):
        x, _, _ = oracle_solution(bt20, b, 20)
        assert rel_err_u0(u20[b], x[:12]) < TOL_U0 and rel_err_u0(U20[b], x) < TOL_U0, b
    eng = _engine(N)
    empty = {k: v[:0] for k, v in bt.items()}
    out = eng.solve(empty["x0"], empty["xref"], empty["contact"], empty["feet"], robot=empty["robot"])
    assert tuple(out.shape) == (0, 12)


@pytest.mark.parametrize("N", [10, 16])
def test_deterministic_and_stream_ordered(N):
    """Repeated launches (the queued classes reset their queues) and other streams
    give bitwise-identical results."""
    import torch
    from mpcqp.synthetic import make_batch
    bt = make_batch(256, N, seed=9, gaits=("trot10", "pace10", "bound8"), robots=("a1",))
    bt["contact"][::7] = 1.0   # some standing robots: every queued class in one call
    eng = _engine(N)
    a = _solve(eng, bt)
    a2 = _solve(eng, bt)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        b = _solve(eng, bt)
    for x, y, z in zip(a, a2, b):
        np.testing.assert_array_equal(x, y)
        np.testing.assert_array_equal(x, z)


def test_full_size_properties():
    """Every bench config's per-GPU shape (2: 1024 x N10, 3: 4096 x N10 mixed, 4: 2048 x
    N16, 5: 8192 x N20 mixed A1/Aliengo with tilted cones; configs 4 and 5 with every
    16th robot standing -- the interior-point class): size-independent properties of
    every solution -- feasibility of every cone row, swing GRFs exactly 0, status OK --
    plus oracle parity on a sample that includes standing robots."""
    from mpcqp.synthetic import make_batch
    mu = 0.7
    for B, N, gaits, robots, tilt in ((1024, 10, ("trot10",), ("a1",), 0.0),
                                      (4096, 10, ("trot10", "pace10", "bound8"), ("a1",), 0.0),
                                      (2048, 16, ("trot10", "pace10", "bound8"), ("a1",), 0.0),
                                      (8192, 20, ("trot10", "pace10", "bound8"), ("a1", "aliengo"), 15.0)):
        bt = make_batch(B, N, seed=2024, gaits=gaits, robots=robots, tilt_deg=tilt)
        if N > 10:
            bt["contact"][::16] = 1.0   # standing (mpc scripts start in Gait.STANDING)
        u0, U, status, iters = _solve(_engine(N), bt)
        assert (status == 0).all(), (N, np.unique(status, return_counts=True))
        f = U.reshape(B, N, 4, 3)
        c = bt["contact"]
        assert np.all(f[c == 0] == 0)
        # cone rows in the robot's own (t1, t2, n) frame
        nrm = bt["robot"][:, 9:12].astype(np.float64)
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        t1 = np.array([1.0, 0.0, 0.0])[None, :] - nrm[:, :1] * nrm
        t1 /= np.linalg.norm(t1, axis=1, keepdims=True)
        t2 = np.cross(nrm, t1)
        fn = np.einsum("bnlk,bk->bnl", f, nrm)
        f1 = np.einsum("bnlk,bk->bnl", f, t1)
        f2 = np.einsum("bnlk,bk->bnl", f, t2)
        tol = 1e-4 * (1.0 + np.abs(f).max(axis=(1, 2, 3)))[:, None, None]
        assert np.all(fn >= -tol) and np.all(fn <= 500.0 + tol)
        assert np.all(np.abs(f1) <= mu * fn + tol) and np.all(np.abs(f2) <= mu * fn + tol)
        # a spread of robots plus the batch's three longest solves (the most degenerate
        # active sets, the launch's tail)
        tail = np.argsort(iters, kind="stable")[-3:].tolist()
        for b in list(range(0, B, B // 8)) + [B // 2 + 1, B - 3] + tail:
            x, _, _ = oracle_solution(bt, b, N)
            assert rel_err_u0(u0[b], x[:12]) < TOL_U0, (N, b, int(iters[b]))
            assert rel_err_u0(U[b], x) < TOL_U0, (N, b, int(iters[b]))


@pytest.mark.parametrize("N", [10, 16])
def test_binding_bounds_and_friction_extremes(N):
    """Per-robot cone parameters at their extremes, in both capacity classes: a
    40 N fz_max (the fz <= ub row binds on 4-10 foot-steps, mpc.py:253-257), low
    and high friction (mu = 0.2 / 1.5, mpc.py:239-245) and a 4x heavier body."""
    from mpcqp.synthetic import make_batch
    bt = make_batch(8, N, seed=31, gaits=("trot10", "pace10", "bound8"), robots=("a1",))
    bt["robot"][0:2, 8] = 40.0
    bt["robot"][2:4, 7] = 0.2
    bt["robot"][4:6, 7] = 1.5
    bt["robot"][6:8, 0] *= 4.0
    u0, U, status, _ = _solve(_engine(N), bt)
    assert (status == 0).all(), status
    bound_rows = 0
    for b in range(8):
        x, _, _ = oracle_solution(bt, b, N)
        assert rel_err_u0(u0[b], x[:12]) < TOL_U0, (b, u0[b], x[:12])
        assert rel_err_u0(U[b], x) < TOL_U0, b
        assert rel_err_u0(U[b], x) < TOL_ACHIEVED, (b, rel_err_u0(U[b], x))
        fz = U[b].reshape(-1, 3)[:, 2]
        assert np.all(fz <= bt["robot"][b, 8] * (1 + 1e-5))
        bound_rows += int(np.sum(np.abs(x.reshape(-1, 3)[:, 2] - bt["robot"][b, 8]) < 1e-6))
    assert bound_rows >= 8   # the case really exercises the upper-bound rows


def test_capacity_class_routing():
    """One N = 16 call reaching every capacity class: n = 96 (class 96), n = 114 and
    126 (class 128), n = 60 (class 64) and standing n = 192 (the interior-point class),
    then twice more (the device queues reset themselves), and with a stance hint the
    batch breaks (the promise is the caller's: the robot beyond it is reported)."""
    from mpcqp.synthetic import make_batch
    N = 16
    bt = make_batch(8, N, seed=41, gaits=("trot10",), robots=("a1",))
    bt["contact"][1, :3, :] = 1.0                  # 3 trot steps made full stance: n = 114
    bt["contact"][2, :5, :] = 1.0                  # n = 126 (the class 128 maximum)
    bt["contact"][3, 10:, :] = 0.0                 # n = 60
    bt["contact"][4] = 1.0                         # standing: n = 192
    ns = 3 * (bt["contact"] > 0).reshape(8, -1).sum(1)
    assert ns[1] > 96 and ns[2] == 126 and ns[3] <= 64 and ns[4] > 126
    eng = _engine(N)
    for _ in range(3):
        u0, U, status, _ = _solve(eng, bt)
        for b in (0, 1, 2, 3, 4, 5):
            assert status[b] == 0, (b, status)
            x, _, _ = oracle_solution(bt, b, N)
            assert rel_err_u0(U[b], x) < TOL_U0, b
    hinted = _engine(N, max_stance=32)             # promises n <= 96: class 128 not launched
    _, _, st, _ = _solve(hinted, bt)
    assert st[1] == 3 and st[2] == 3 and st[4] == 3
    assert all(st[b] == 0 for b in (0, 3, 5, 6, 7))


def test_class64_capacity_boundary():
    """Both sides of class 64's capacity (n = 60 / 63 / 66 at N = 10: 20 / 21 / 22 stance
    foot-steps), with and without a stance range that launches the first possible class
    directly, match the oracle."""
    from mpcqp.synthetic import make_batch
    N = 10
    bt = make_batch(6, N, seed=63, gaits=("trot10",), robots=("a1",))
    bt["contact"][0] = 0.0
    bt["contact"][0].reshape(-1)[:21] = 1.0        # n = 63
    bt["contact"][1] = 0.0
    bt["contact"][1].reshape(-1)[:20] = 1.0        # n = 60
    bt["contact"][2] = 0.0
    bt["contact"][2].reshape(-1)[::2] = 1.0        # n = 60, alternating feet
    bt["contact"][3] = 0.0
    bt["contact"][3].reshape(-1)[:22] = 1.0        # n = 66: class 96
    ns = 3 * (bt["contact"] > 0).reshape(6, -1).sum(1)
    assert ns[0] == 63 and ns[1] == 60 and ns[2] == 60 and ns[3] == 66
    for rng in ((0, 0), (20, 21), (21, 21), (22, 22)):
        eng = _engine(N)
        eng.set_stance_range(*rng)
        sel = [b for b in range(6) if rng == (0, 0) or rng[0] <= ns[b] // 3 <= rng[1]]
        sub = {k: v[sel] for k, v in bt.items()}
        u0, U, status, _ = _solve(eng, sub)
        assert (status == 0).all(), (rng, status)
        for i, b in enumerate(sel):
            x, _, _ = oracle_solution(bt, b, N)
            assert rel_err_u0(U[i], x) < TOL_ACHIEVED, (rng, b, rel_err_u0(U[i], x))


def test_two_streams_no_host_sync():
    """One context, two streams, no host synchronisation between the calls: each
    stream has its own device queues, so robots of the queued classes (N = 16 trot /
    pace / bound -> class 96, standing -> the interior-point class) never mix."""
    import torch
    from mpcqp.synthetic import make_batch
    N = 16
    eng = _engine(N)
    bts = []
    for seed in (51, 52):
        bt = make_batch(96, N, seed=seed, gaits=("trot10", "pace10", "bound8"), robots=("a1",))
        bt["contact"][seed % 5::9] = 1.0
        bts.append(bt)
    dev = torch.device("cuda:0")
    ins = [{k: torch.as_tensor(v).to(dev) for k, v in bt.items()} for bt in bts]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for s, t in zip(streams, ins):
        with torch.cuda.stream(s):
            outs.append(eng.solve(t["x0"], t["xref"], t["contact"], t["feet"], robot=t["robot"],
                                  return_all=True, stream=s))
    torch.cuda.synchronize()
    for bt, res in zip(bts, outs):
        status = res.status.cpu().numpy()
        U = res.U.cpu().numpy().reshape(len(bt["x0"]), -1)
        assert (status == 0).all(), status
        for b in range(0, len(bt["x0"]), 7):
            x, _, _ = oracle_solution(bt, b, N)
            assert rel_err_u0(U[b], x) < TOL_U0, b


def test_interior_point_throughput_layout():
    """An all-standing batch larger than three robots per CU, promised as such
    (mpcqp_set_stance_range(4N, 4N)): the interior-point class takes it directly in its
    throughput layout (four robots per CU, M_k in the global slot) -- every status OK and
    sampled robots against the oracle; the same robots through the latency layout (a small
    batch) agree to the interior-point guard."""
    import torch
    from mpcqp.synthetic import make_batch
    N = 16
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    B = 3 * ncu + 16
    bt = make_batch(B, N, seed=910, gaits=("trot10",), robots=("a1", "aliengo"), tilt_deg=5.0)
    bt["contact"][:] = 1.0
    eng = _engine(N)
    eng.set_stance_range(4 * N, 4 * N)
    u0, U, status, iters = _solve(eng, bt)
    assert (status == 0).all(), np.unique(status, return_counts=True)
    assert (iters > 0).all()
    pick = [0, 1, B // 2, B - 2, B - 1]
    small = {k: v[pick] for k, v in bt.items()}
    u0s, Us, sts, _ = _solve(_engine(N), small)
    assert (sts == 0).all()
    for j, b in enumerate(pick):
        x, _, _ = oracle_solution(bt, b, N)
        assert max(rel_err_u0(u0[b], x[:12]), rel_err_u0(U[b], x)) < TOL_ACHIEVED_IPM, b
        assert rel_err_u0(U[b], Us[j].astype(np.float64)) < TOL_ACHIEVED_IPM, b


def test_interior_point_standing_fleet_tail():
    """Config 4's synthetic fleet all standing (2 048 robots, the bench's `--standing-every 1`
    batch): every status OK, no robot above 18 factorisations (round 6: the Tapia polish set,
    two corrections after an interior-point polish and the 0.98 step fraction; the slowest
    robots of this batch took 22 and 21 before), and those two robots plus a sample against
    the oracle."""
    from mpcqp.synthetic import make_batch
    N = 16
    bt = make_batch(2048, N, seed=1000, gaits=("trot10", "pace10", "bound8"), robots=("a1",))
    bt["contact"][:] = 1.0
    eng = _engine(N)
    eng.set_stance_range(4 * N, 4 * N)
    u0, U, status, iters = _solve(eng, bt)
    assert (status == 0).all(), np.unique(status, return_counts=True)
    assert iters.max() <= 18, (int(iters.max()), int(np.argmax(iters)))
    assert iters.mean() < 11.5, iters.mean()
    for b in (1083, 231, 0, 1024, 2047):
        x, _, _ = oracle_solution(bt, b, N)
        assert max(rel_err_u0(u0[b], x[:12]), rel_err_u0(U[b], x)) < TOL_ACHIEVED_IPM, b


def test_queue_set_eviction_beyond_eight_streams():
    """A context keeps queues for 8 streams; solves round-robin over 11 streams make the
    9th-11th take over the least recently used sets (after waiting on their last solve's
    event, with their buffers reused) -- every stream's batch (trot / pace / bound routed
    to class 96, standing robots to the interior-point class) still gives the oracle's
    optimum, over two rounds so reused sets are used again."""
    import torch
    from mpcqp.synthetic import make_batch
    N = 16
    eng = _engine(N)
    dev = torch.device("cuda:0")
    streams = [torch.cuda.Stream() for _ in range(11)]
    bts = []
    for i in range(len(streams)):
        bt = make_batch(24, N, seed=700 + i, gaits=("trot10", "pace10", "bound8"), robots=("a1",))
        bt["contact"][i % 4::6] = 1.0
        bts.append(bt)
    ins = [{k: torch.as_tensor(v).to(dev) for k, v in bt.items()} for bt in bts]
    torch.cuda.synchronize()
    for rnd in range(2):
        outs = []
        for s, t in zip(streams, ins):
            with torch.cuda.stream(s):
                outs.append(eng.solve(t["x0"], t["xref"], t["contact"], t["feet"], robot=t["robot"],
                                      return_all=True, stream=s))
        torch.cuda.synchronize()
        for i, (bt, res) in enumerate(zip(bts, outs)):
            status = res.status.cpu().numpy()
            assert (status == 0).all(), (rnd, i, status)
            U = res.U.cpu().numpy().reshape(len(bt["x0"]), -1)
            for b in (i % 4, 5, 23):
                x, _, _ = oracle_solution(bt, b, N)
                assert rel_err_u0(U[b], x) < TOL_U0, (rnd, i, b)


@pytest.mark.parametrize("N", [10, 16, 20])
def test_random_contact_patterns_every_class(N):
    """Arbitrary (not gait-table) contact patterns with per-robot mu, fz_max and tilted
    cone normals: stance counts from 0 to 4N, so one call routes robots to every
    capacity class (64 / 96 / 128 and the interior-point class for n > 128 at
    N = 16 / 20) -- each robot's u0 and U against the float64 oracle."""
    from mpcqp.params import R_FZMAX, R_MU, R_NX, R_NZ
    from mpcqp.synthetic import make_batch
    B = 40
    rng = np.random.default_rng(100 + N)
    bt = make_batch(B, N, seed=200 + N, gaits=("trot10", "pace10", "bound8"), robots=("a1", "aliengo"),
                    tilt_deg=20.0)
    density = rng.uniform(0.05, 1.0, size=(B, 1, 1))
    bt["contact"] = (rng.random((B, N, 4)) < density).astype(np.float32)
    bt["contact"][0] = 1.0   # standing over the whole horizon (n = 12 N)
    bt["contact"][1] = 0.0   # flight over the whole horizon (n = 0)
    bt["robot"][:, R_MU] = rng.uniform(0.2, 1.0, B).astype(np.float32)
    bt["robot"][:, R_FZMAX] = rng.uniform(120.0, 600.0, B).astype(np.float32)
    u0, U, status, _ = _solve(_engine(N), bt)
    assert (status == 0).all(), status
    stance = bt["contact"].reshape(B, -1).sum(1)
    assert stance.max() == 4 * N and stance.min() == 0
    worst, worst_ipm = 0.0, 0.0
    for b in range(B):
        x, _, _ = oracle_solution(bt, b, N)
        assert rel_err_u0(u0[b], x[:12]) < TOL_U0, (b, int(stance[b]), u0[b], x[:12])
        e = max(rel_err_u0(u0[b], x[:12]), rel_err_u0(U[b], x))
        if 3 * stance[b] > 128:
            worst_ipm = max(worst_ipm, e)
        else:
            worst = max(worst, e)
        assert rel_err_u0(U[b], x) < TOL_U0, (b, int(stance[b]))
    assert worst < TOL_ACHIEVED, worst
    assert worst_ipm < TOL_ACHIEVED_IPM, worst_ipm
    assert np.all(U[1] == 0) and np.all(u0[1] == 0)
    assert bt["robot"][:, R_NX:R_NZ + 1].shape == (B, 3)


@pytest.mark.parametrize("N", [24, 32])
def test_long_horizons_interior_point(N):
    """Horizons beyond the dense classes' 20-stage layouts (LinearMpcConfig.horizon is a
    free value, linear_mpc_configs.py:11; MPCQP_MAX_HORIZON = 32): the interior-point class
    takes the whole batch -- gait-table trot / pace / bound schedules, a standing and a
    sparse robot (n well below 128) and a flight schedule -- each robot's u0 and U against
    the float64 oracle at the contract and the interior-point precision guard."""
    from mpcqp.synthetic import make_batch
    B = 10 if N == 32 else 12
    rng = np.random.default_rng(300 + N)
    bt = make_batch(B, N, seed=400 + N, gaits=("trot10", "pace10", "bound8"), robots=("a1", "aliengo"),
                    tilt_deg=10.0)
    bt["contact"][0] = 1.0                                              # standing: n = 12 N
    bt["contact"][1] = (rng.random((N, 4)) < 0.2).astype(np.float32)    # sparse: n < 128
    bt["contact"][2] = 0.0                                              # flight: n = 0
    u0, U, status, iters = _solve(_engine(N), bt)
    assert (status == 0).all(), status
    worst = 0.0
    for b in range(B):
        x, _, _ = oracle_solution(bt, b, N)
        e = max(rel_err_u0(u0[b], x[:12]), rel_err_u0(U[b], x))
        assert e < TOL_U0, (b, e)
        worst = max(worst, e)
    assert worst < TOL_ACHIEVED_IPM, worst
    assert np.all(U[2] == 0) and np.all(u0[2] == 0)
    assert iters[0] > 0   # Newton factorisations: the interior-point class solved it


@pytest.mark.parametrize("N", [16, 24])
def test_warm_start_interior_point(N):
    """mpcqp_set_warm_start: a fleet solved tick after tick (x0 drifting by a few mm / mrad
    per tick) with each robot's previous active set remembered -- every tick's u0 and U
    against the float64 oracle, statuses OK, and the warm interior-point robots needing
    fewer Newton factorisations than the cold engine.  Then the memory is scrambled
    (every robot handed another robot's set): still the oracle's optimum, since a set
    that fails the KKT check is corrected or abandoned for the cold start."""
    import torch
    from mpcqp.synthetic import make_batch
    B = 8
    bt = make_batch(B, N, seed=500 + N, gaits=("trot10", "pace10", "bound8"), robots=("a1", "aliengo"))
    bt["contact"][:6] = 1.0   # six standing robots (the interior-point class), two gait robots
    warm, cold = _engine(N), _engine(N)
    mem = warm.set_warm_start(B)
    assert mem.shape == (B, 128) and int(mem.sum()) == 0
    rng = np.random.default_rng(600 + N)
    fw, fc = [], []
    for tick in range(4):
        if tick:
            bt["x0"][:, :12] += rng.normal(0.0, 2e-3, size=(B, 12)).astype(np.float32)
        u0, U, status, iters = _solve(warm, bt)
        _, _, status_c, iters_c = _solve(cold, bt)
        assert (status == 0).all() and (status_c == 0).all(), (tick, status, status_c)
        for b in range(B):
            x, _, _ = oracle_solution(bt, b, N)
            e = max(rel_err_u0(u0[b], x[:12]), rel_err_u0(U[b], x))
            assert e < TOL_ACHIEVED_IPM, (tick, b, e)
        if tick:
            fw.append(iters[:6].sum())
            fc.append(iters_c[:6].sum())
        m = mem.cpu().numpy()
        assert np.all(m[:6, :4 * N] & 0x80) and np.all(m[:, 4 * N:] == 0), tick   # verified sets remembered
    assert sum(fw) < sum(fc), (fw, fc)
    # scrambled memory: robot b gets robot b + 1's set
    mem.copy_(torch.roll(mem, 1, dims=0))
    bt["x0"][:, :12] += rng.normal(0.0, 2e-2, size=(B, 12)).astype(np.float32)
    u0, U, status, _ = _solve(warm, bt)
    assert (status == 0).all(), status
    for b in range(B):
        x, _, _ = oracle_solution(bt, b, N)
        assert max(rel_err_u0(u0[b], x[:12]), rel_err_u0(U[b], x)) < TOL_ACHIEVED_IPM, b
    warm.set_warm_start(0)


def test_stance_range_direct_classes():
    """mpcqp_set_stance_range: when the range rules out the smaller classes, the first
    possible class takes the batch directly -- the same kernels and arithmetic as the
    routed path (bitwise), and robots below the range are still solved (by a larger
    class) to the oracle's tolerance."""
    from mpcqp.synthetic import make_batch
    N = 16
    bt = make_batch(12, N, seed=21, gaits=("trot10",), robots=("a1", "aliengo"))   # 32 stance steps: class 96
    bt["contact"][::4] = 1.0                                                      # 64: interior point
    eng = _engine(N)
    ref = _solve(eng, bt)
    eng.set_stance_range(32, 64)   # class 96 direct, the interior-point class queued
    got = _solve(eng, bt)
    for x, y in zip(ref, got):
        np.testing.assert_array_equal(x, y)
    stand = {k: v[::4].copy() for k, v in bt.items()}
    eng.set_stance_range(0, 0)
    ref_s = _solve(eng, stand)
    eng.set_stance_range(64, 64)   # the interior-point class direct
    got_s = _solve(eng, stand)
    for x, y in zip(ref_s, got_s):
        np.testing.assert_array_equal(x, y)
    # robots below the range's minimum: N = 10 trot (20 stance steps) through class 96 direct
    bt10 = make_batch(6, 10, seed=22, gaits=("trot10",), robots=("a1",))
    eng10 = _engine(10)
    eng10.set_stance_range(25, 40)
    u0, U, status, _ = _solve(eng10, bt10)
    assert (status == 0).all(), status
    for b in range(6):
        x, _, _ = oracle_solution(bt10, b, 10)
        assert rel_err_u0(u0[b], x[:12]) < TOL_U0 and rel_err_u0(U[b], x) < TOL_U0, b


def test_stance_range_rejects_impossible_minimum_and_empty_ipm_robot():
    """a min_stance above 4 N (no schedule has that many stance foot-steps)
    is rejected instead of silently launching nothing; a robot with no stance
    foot-step sent straight to the interior-point class (a broken promise) returns
    U = 0 with status OK, as the dense classes do, instead of 60 NaN iterations."""
    from mpcqp import _lib
    from mpcqp.synthetic import make_batch
    eng = _engine(10)
    with pytest.raises(_lib.MpcqpError, match="4 \\* horizon"):
        eng.set_stance_range(41, 0)
    eng.set_stance_range(40, 0)   # every foot in stance at every step: accepted
    N = 16
    bt = make_batch(3, N, seed=5, gaits=("trot10",), robots=("a1",))
    bt["contact"][1] = 0.0        # robot 1: flight at every step
    eng16 = _engine(N)
    eng16.set_stance_range(43, 64)   # the interior-point class takes the batch directly
    u0, U, status, iters = _solve(eng16, bt)
    assert (status == 0).all(), status
    assert np.all(U[1] == 0) and np.all(u0[1] == 0) and iters[1] == 0
    for b in (0, 2):
        x, _, _ = oracle_solution(bt, b, N)
        assert rel_err_u0(u0[b], x[:12]) < TOL_U0, b


def _full_weights(seed, cross_leg_r=False):
    """A symmetric positive-semidefinite Q coupling the state components (the reference's
    diagonal scaled by a correlation matrix, |rho| <= 0.4: the weighting keeps the
    reference's scale, so the float32 condensing of mpc.py:213-230 perturbs the optimum
    as little as with the diagonal) and a leg-block R (or one with cross-leg terms)."""
    from mpcqp.params import Q_DIAG, R_DIAG
    rng = np.random.default_rng(seed)
    C = np.eye(13)
    for _ in range(12):
        i, j = rng.choice(12, size=2, replace=False)   # state 12 (gravity) keeps weight 0
        C[i, j] = C[j, i] = rng.uniform(-0.4, 0.4)
    w, V = np.linalg.eigh(C)
    C = V @ np.diag(np.maximum(w, 0.05)) @ V.T           # positive definite
    d = np.sqrt(np.diag(C))
    C = C / np.outer(d, d)
    sq = np.sqrt(np.asarray(Q_DIAG, np.float64))
    Q = np.outer(sq, sq) * C
    R = np.diag(R_DIAG).copy()
    for leg in range(4):
        S = rng.uniform(-0.3, 0.3, size=(3, 3))
        R[3 * leg:3 * leg + 3, 3 * leg:3 * leg + 3] += 1e-5 * (S @ S.T)
    if cross_leg_r:
        R[1, 7] = R[7, 1] = 3e-6
    return 0.5 * (Q + Q.T), 0.5 * (R + R.T)


@pytest.mark.parametrize("N", [10, 16, 20])
def test_full_weights_match_oracle(N):
    """General (non-diagonal) Q and leg-block R (mpc.py:50,52 take full matrices,
    mpcqp_set_weights): random contact patterns route robots to every dense class and,
    at N = 16 / 20, the interior-point class -- u0 and U against the float64 oracle
    formulated with the same full Qbar = kron(I_N, Q), Rbar = kron(I_N, R)."""
    from mpcqp.synthetic import make_batch
    B = 24
    rng = np.random.default_rng(300 + N)
    bt = make_batch(B, N, seed=400 + N, gaits=("trot10", "pace10", "bound8"), robots=("a1", "aliengo"),
                    tilt_deg=15.0)
    density = rng.uniform(0.05, 1.0, size=(B, 1, 1))
    bt["contact"] = (rng.random((B, N, 4)) < density).astype(np.float32)
    bt["contact"][0] = 1.0
    Q, R = _full_weights(N)
    eng = _engine(N, Q=Q, R=R)
    u0, U, status, _ = _solve(eng, bt)
    assert (status == 0).all(), status
    stance = bt["contact"].reshape(B, -1).sum(1)
    worst, worst_ipm = 0.0, 0.0
    for b in range(B):
        x, _, _ = oracle_solution(bt, b, N, Q=Q, R=R)
        e = max(rel_err_u0(u0[b], x[:12]), rel_err_u0(U[b], x))
        assert e < TOL_U0, (b, int(stance[b]), e)
        if 3 * stance[b] > 128:
            worst_ipm = max(worst_ipm, e)
        else:
            worst = max(worst, e)
    assert worst < TOL_ACHIEVED, worst
    assert worst_ipm < TOL_ACHIEVED_IPM, worst_ipm
    # back to the diagonal weights: the fast path again, bitwise as a fresh engine
    from mpcqp.params import Q_DIAG, R_DIAG
    eng.set_weights(Q_DIAG, R_DIAG)
    got = _solve(eng, bt)
    ref = _solve(_engine(N), bt)
    for a, c in zip(got, ref):
        np.testing.assert_array_equal(a, c)


@pytest.mark.parametrize("N,B,first", [(10, 3000, False), (16, 600, True), (20, 300, True)])
def test_dispatch_order_full_weights(N, B, first):
    """The full-weight kernel instantiations (mpcqp_set_weights) under the dispatch order:
    class 64 sorting its XCD ranges, classes 96 / 128 taking the batch directly -- bitwise
    equal to batch order, and on the oracle's optimum."""
    from mpcqp.synthetic import make_batch
    bt = make_batch(B, N, seed=950 + N, gaits=("trot10", "pace10", "bound8"), robots=("a1",))
    stance = (bt["contact"] > 0).reshape(B, -1).sum(1)
    Q, R = _full_weights(N)
    out = []
    for mode in (0, 1):
        eng = _engine(N, Q=Q, R=R)
        if first:
            eng.set_stance_range(int(stance.min()), int(stance.max()))
        eng.set_order(mode)
        out.append(_solve(eng, bt))
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(a, b)
    assert (out[1][2] == 0).all()
    x, _, _ = oracle_solution(bt, B - 1, N, Q=Q, R=R)
    assert rel_err_u0(out[1][0][B - 1], x[:12]) < TOL_U0


def test_full_weights_cross_leg_r_and_validation():
    """A cross-leg R entry: the dense classes and the interior-point class (its XR
    instantiations: 12 x 12 stage weights) solve it (oracle parity).  The C ABI rejects an
    asymmetric or non-finite weight with MPCQP_ERR_ARG and keeps the previous weights."""
    import ctypes
    from mpcqp import _lib
    from mpcqp.synthetic import make_batch
    N = 16
    B = 8
    bt = make_batch(B, N, seed=77, gaits=("trot10",), robots=("a1",))
    bt["contact"][::4] = 1.0   # robots 0, 4 standing: n = 192, the interior-point class
    Q, R = _full_weights(5, cross_leg_r=True)
    eng = _engine(N, Q=Q, R=R)
    u0, U, status, _ = _solve(eng, bt)
    assert (status == 0).all(), status
    for b in range(B):
        x, _, _ = oracle_solution(bt, b, N, Q=Q, R=R)
        tol = TOL_ACHIEVED_IPM if b % 4 == 0 else TOL_ACHIEVED   # robots 0, 4: interior point
        assert max(rel_err_u0(u0[b], x[:12]), rel_err_u0(U[b], x)) < tol, b
    def set_raw(ctx, q, r):
        return int(eng.lib.mpcqp_set_weights(ctx, np.ascontiguousarray(q).ctypes.data,
                                             np.ascontiguousarray(r).ctypes.data))
    bad = Q.copy()
    bad[0, 1] += 1.0
    assert set_raw(eng._ctx, bad, R) == _lib.ERR_ARG
    nan = Q.copy()
    nan[3, 3] = np.nan
    assert set_raw(eng._ctx, nan, R) == _lib.ERR_ARG
    inf = R.copy()
    inf[2, 2] = np.inf
    assert set_raw(eng._ctx, Q, inf) == _lib.ERR_ARG
    assert set_raw(ctypes.c_void_p(0), Q, R) == _lib.ERR_ARG
    again = _solve(eng, bt)   # the previous (valid) weights still in force
    np.testing.assert_array_equal(again[0], u0)
    # NULL keeps the current matrix whole: (Q_full, R) then (NULL, R) solves as (Q_full, R)
    null = ctypes.c_void_p(0)
    assert int(eng.lib.mpcqp_set_weights(eng._ctx, null, np.ascontiguousarray(R).ctypes.data)) == 0
    kept = _solve(eng, bt)
    np.testing.assert_array_equal(kept[0], u0)
    assert int(eng.lib.mpcqp_set_weights(eng._ctx, np.ascontiguousarray(Q).ctypes.data, null)) == 0
    np.testing.assert_array_equal(_solve(eng, bt)[0], u0)


def _cross_leg_weights(seed):
    """The full Q of _full_weights and an R coupling every pair of legs: the reference's
    diagonal scaled by a dense random correlation matrix (SPD, every cross-leg block non-zero)."""
    from mpcqp.params import R_DIAG
    Q, _ = _full_weights(seed)
    rng = np.random.default_rng(seed + 1)
    A = rng.standard_normal((12, 12))
    C = A @ A.T / 12.0 + 0.5 * np.eye(12)
    d = np.sqrt(np.diag(C))
    C = C / np.outer(d, d)
    sq = np.sqrt(np.asarray(R_DIAG, np.float64))
    R = np.outer(sq, sq) * C
    return Q, 0.5 * (R + R.T)


@pytest.mark.parametrize("N", [16, 20, 24, 32])
def test_cross_leg_r_interior_point(N):
    """A dense cross-leg R (mpc.py:51-52 take any symmetric R) in the interior-point class: the
    XR instantiations' 12 x 12 stage weights W_k = (Rh + blockdiag G^T D G)^-1 and the polish's
    P (P Rh P + I - P)^-1 P.  Standing, near-standing and dense random schedules (n > 128 at
    N = 16 / 20; every robot at N > 20) against the float64 oracle with the same
    Rbar = kron(I_N, R); the dense-class robots of the batch too."""
    from mpcqp.synthetic import make_batch
    B = 8 if N <= 20 else 5
    bt = make_batch(B, N, seed=500 + N, gaits=("trot10", "pace10", "bound8"), robots=("a1", "aliengo"),
                    tilt_deg=10.0)
    rng = np.random.default_rng(600 + N)
    bt["contact"][:] = (rng.random((B, N, 4)) < rng.uniform(0.75, 1.0, size=(B, 1, 1))).astype(np.float32)
    bt["contact"][0] = 1.0                      # standing
    bt["contact"][1] = 1.0
    bt["contact"][1, N // 2:, 2] = 0.0          # near standing
    Q, R = _cross_leg_weights(N)
    assert np.abs(R[:3, 3:]).min() > 0.0
    eng = _engine(N, Q=Q, R=R)
    u0, U, status, iters = _solve(eng, bt)
    assert (status == 0).all(), status
    stance = bt["contact"].reshape(B, -1).sum(1)
    for b in range(B):
        x, _, _ = oracle_solution(bt, b, N, Q=Q, R=R)
        e = max(rel_err_u0(u0[b], x[:12]), rel_err_u0(U[b], x))
        tol = TOL_ACHIEVED_IPM if (3 * stance[b] > 128 or N > 20) else TOL_ACHIEVED
        assert e < tol, (b, int(stance[b]), e)
    # the warm start's polish (mpcqp_set_warm_start) takes the same stage weights: a second
    # tick from the remembered sets reaches the same optimum
    eng.set_warm_start(B)
    _solve(eng, bt)
    w = _solve(eng, bt)
    assert (w[2] == 0).all()
    for b in range(B):
        assert rel_err_u0(w[0][b], u0[b]) < 2 * TOL_ACHIEVED_IPM, b
