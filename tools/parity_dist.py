"""Diagnostic: per-robot achieved precision (u0 and U, norm-wise relative) of the
random-contact parity case (tests/test_gpu_parity.py) by stance count and class."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pympc-quadruped_amd"), ROOT, os.path.join(ROOT, "tests")]


def main():
    from helpers import oracle_solution, rel_err_u0
    from mpcqp import LinearMpc
    from mpcqp.params import R_FZMAX, R_MU
    from mpcqp.synthetic import make_batch
    for N in (10, 16, 20):
        B = 40
        rng = np.random.default_rng(100 + N)
        bt = make_batch(B, N, seed=200 + N, gaits=("trot10", "pace10", "bound8"), robots=("a1", "aliengo"),
                        tilt_deg=20.0)
        density = rng.uniform(0.05, 1.0, size=(B, 1, 1))
        bt["contact"] = (rng.random((B, N, 4)) < density).astype(np.float32)
        bt["contact"][0] = 1.0
        bt["contact"][1] = 0.0
        bt["robot"][:, R_MU] = rng.uniform(0.2, 1.0, B).astype(np.float32)
        bt["robot"][:, R_FZMAX] = rng.uniform(120.0, 600.0, B).astype(np.float32)
        eng = LinearMpc(horizon=N, robot="a1")
        res = eng.solve(bt["x0"], bt["xref"], bt["contact"], bt["feet"], robot=bt["robot"], return_all=True)
        u0 = res.u0.cpu().numpy()
        U = res.U.cpu().numpy().reshape(B, -1)
        it = res.iterations.cpu().numpy()
        st = res.status.cpu().numpy()
        stance = bt["contact"].reshape(B, -1).sum(1)
        rows = []
        for b in range(B):
            x, _, _ = oracle_solution(bt, b, N)
            rows.append((rel_err_u0(u0[b], x[:12]), rel_err_u0(U[b], x), int(3 * stance[b]), int(it[b]), int(st[b])))
        rows.sort(key=lambda r: -max(r[0], r[1]))
        print(f"N={N}: worst 6 (u0 err, U err, n, iters, status):")
        for r in rows[:6]:
            print("   %.2e %.2e n=%d it=%d st=%d" % r)


if __name__ == "__main__":
    main()
