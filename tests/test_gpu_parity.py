"""GPU parity: the HIP engine vs the float64 oracle and the reference's own
fixtures, on identical inputs (-m gpu).  Every call goes through the C ABI
(libmpcqp.so via mpcqp.LinearMpc)."""
import os

import numpy as np
import pytest

from helpers import oracle_solution, rel_err_u0

TOL_U0 = 1e-4   # north_star: GRF within 1e-4 relative, norm-wise ||du0||_inf / ||u0*||_inf
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
NV_MAX = 64     # stance variables handled by this build's kernel (n = 3 * #stance)

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
])
def test_u0_matches_oracle(N, gaits, robots, tilt):
    from mpcqp.synthetic import make_batch
    B = 24
    bt = make_batch(B, N, seed=11, gaits=gaits, robots=robots, tilt_deg=tilt)
    u0, U, status, _ = _solve(_engine(N), bt)
    assert (status == 0).all(), status
    for b in range(B):
        x, _, _ = oracle_solution(bt, b, N)
        assert rel_err_u0(u0[b], x[:12]) < TOL_U0, (b, u0[b], x[:12])
        assert rel_err_u0(U[b], x) < TOL_U0, b


@pytest.mark.parametrize("N", [10, 16, 20])
def test_reference_golden_fixtures(N):
    """u* of QPs built by the reference's own functions (tests/golden/make_golden.py)."""
    z = np.load(os.path.join(GOLDEN, f"formulation_N{N}.npz"), allow_pickle=False)
    bt = {k: z[k] for k in ("x0", "xref", "contact", "feet", "robot")}
    u0, U, status, _ = _solve(_engine(N), bt)
    n_eff = 3 * (bt["contact"] > 0).reshape(len(bt["x0"]), -1).sum(1)
    checked = 0
    for b in range(len(bt["x0"])):
        if n_eff[b] > NV_MAX:
            assert status[b] == 3   # MPCQP_STATUS_TOO_LARGE: reported, never silently wrong
            continue
        assert status[b] == 0
        assert rel_err_u0(u0[b], z["u_star"][b][:12]) < TOL_U0, (b, u0[b], z["u_star"][b][:12])
        assert rel_err_u0(U[b], z["u_star"][b]) < TOL_U0
        checked += 1
    assert N > 10 or checked >= 8


def test_edge_cases():
    from mpcqp.synthetic import make_batch
    N = 10
    bt = make_batch(6, N, seed=5, gaits=("trot10",), robots=("a1",))
    bt["contact"][0] = 0.0                         # flight phase: every GRF is 0
    bt["xref"][1, 3, 4] = np.nan                   # non-finite input
    bt["contact"][2, :, :] = 1.0                   # standing: n = 120 > this build's 64
    bt["contact"][3, 1:, :] = 0.0                  # single step of stance
    bt["contact"][3, 0, :] = 1.0
    u0, U, status, iters = _solve(_engine(N), bt)
    assert status[0] == 0 and np.all(u0[0] == 0) and np.all(U[0] == 0)
    assert status[1] == 4 and np.all(u0[1] == 0)
    assert status[2] == 3
    assert status[3] == 0 and np.all(U[3][12:] == 0)
    x, _, _ = oracle_solution(bt, 3, N)
    assert rel_err_u0(u0[3], x[:12]) < TOL_U0
    for b in (4, 5):
        x, _, _ = oracle_solution(bt, b, N)
        assert status[b] == 0 and rel_err_u0(u0[b], x[:12]) < TOL_U0
    eng = _engine(N)
    empty = {k: v[:0] for k, v in bt.items()}
    out = eng.solve(empty["x0"], empty["xref"], empty["contact"], empty["feet"], robot=empty["robot"])
    assert tuple(out.shape) == (0, 12)


def test_deterministic_and_stream_ordered():
    import torch
    from mpcqp.synthetic import make_batch
    bt = make_batch(256, 10, seed=9, gaits=("trot10", "pace10", "bound8"), robots=("a1",))
    eng = _engine(10)
    a = _solve(eng, bt)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        b = _solve(eng, bt)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_full_size_properties():
    """B = 1024 (config 2) and 4096 (config 3): size-independent properties of every
    solution -- feasibility of every cone row, swing GRFs exactly 0, status OK --
    plus oracle parity on a sample."""
    from mpcqp.synthetic import make_batch
    for B, gaits in ((1024, ("trot10",)), (4096, ("trot10", "pace10", "bound8"))):
        bt = make_batch(B, 10, seed=2024, gaits=gaits, robots=("a1",))
        u0, U, status, iters = _solve(_engine(10), bt)
        assert (status == 0).all()
        f = U.reshape(B, 10, 4, 3)
        c = bt["contact"]
        assert np.all(f[c == 0] == 0)
        fx, fy, fz = f[..., 0], f[..., 1], f[..., 2]
        mu = 0.7
        tol = 1e-4 * (1.0 + np.abs(f).max(axis=(1, 2, 3)))[:, None, None]
        assert np.all(fz >= -tol) and np.all(fz <= 500.0 + tol)
        assert np.all(np.abs(fx) <= mu * fz + tol) and np.all(np.abs(fy) <= mu * fz + tol)
        for b in range(0, B, B // 8):
            x, _, _ = oracle_solution(bt, b, 10)
            assert rel_err_u0(u0[b], x[:12]) < TOL_U0
