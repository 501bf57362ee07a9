"""CPU: the compiled restatement of the reference's formulate + solve
(oracle/cpu_mpc.cpp, bench.py's cpu_baseline) against the reference-built golden
optima and the Python oracle, every horizon, standing schedules included."""
import os

import numpy as np
import pytest

from helpers import oracle_solution, rel_err_u0

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("N", [10, 16, 20])
def test_cpu_port_matches_reference_golden(N):
    from oracle import cpu_port
    z = np.load(os.path.join(GOLDEN, f"formulation_N{N}.npz"), allow_pickle=False)
    bt = {k: z[k] for k in ("x0", "xref", "contact", "feet", "robot")}
    U, it, tf, ts = cpu_port.solve_batch(bt, N, threads=2)
    assert (it >= 0).all()
    for b in range(len(U)):
        assert rel_err_u0(U[b], z["u_star"][b]) < 1e-5, b
    assert tf > 0 and ts > 0


def test_cpu_port_matches_oracle_tilted_mixed():
    from oracle import cpu_port
    from mpcqp.synthetic import make_batch
    N = 10
    bt = make_batch(12, N, seed=8, gaits=("trot10", "pace10", "bound8"), robots=("a1", "aliengo"), tilt_deg=15.0)
    bt["robot"][0, 8] = 40.0     # binding fz_max
    bt["robot"][1, 7] = 0.2      # low friction
    U, it, _, _ = cpu_port.solve_batch(bt, N)
    for b in range(12):
        x, _, _ = oracle_solution(bt, b, N)
        assert rel_err_u0(U[b], x) < 1e-5, b
