"""GPU parity: HIP engine vs the float64 oracle on identical inputs (-m gpu)."""
import numpy as np
import pytest

from helpers import oracle_solution, rel_err_u0

TOL_U0 = 1e-4   # north_star: GRF within 1e-4 relative (norm-wise, fp32 output)

pytestmark = pytest.mark.gpu


def _engine(N, **kw):
    from mpcqp import LinearMpc
    return LinearMpc(horizon=N, robot="a1", **kw)


@pytest.mark.parametrize("N,gaits,robots", [
    (10, ("trot10",), ("a1",)),
    (10, ("trot10", "pace10", "bound8"), ("a1", "aliengo")),
])
def test_u0_matches_oracle(N, gaits, robots):
    from mpcqp.synthetic import make_batch
    B = 24
    bt = make_batch(B, N, seed=11, gaits=gaits, robots=robots)
    eng = _engine(N)
    res = eng.solve(bt["x0"], bt["xref"], bt["contact"], bt["feet"], robot=bt["robot"], return_all=True)
    u0 = res.u0.cpu().numpy()
    U = res.U.cpu().numpy().reshape(B, -1)
    status = res.status.cpu().numpy()
    errs = []
    for b in range(B):
        x, _, _ = oracle_solution(bt, b, N)
        errs.append(rel_err_u0(u0[b], x[:12]))
        assert rel_err_u0(U[b], x) < TOL_U0, (b, np.abs(U[b] - x).max())
    assert (status == 0).all(), status
    assert max(errs) < TOL_U0, errs
