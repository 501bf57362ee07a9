"""Diagnostic (round 6): the interior-point class under an R coupling every pair of legs (the XR
instantiations' 12 x 12 stage weights) -- achieved u0 / U precision against the float64 oracle
and factorisation counts, next to the same robots with the leg-block part of that R only.
  python tools/xr_stats.py [N ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pympc-quadruped_amd"), ROOT, os.path.join(ROOT, "tests")]


def main():
    import torch
    from mpcqp import LinearMpc
    from mpcqp.synthetic import make_batch
    from mpcqp.params import Q_DIAG, R_DIAG
    from helpers import oracle_solution, rel_err_u0
    A = np.random.default_rng(12).standard_normal((12, 12))
    Cr = A @ A.T / 12.0 + 0.5 * np.eye(12)
    dr = np.sqrt(np.diag(Cr))
    sq = np.sqrt(np.asarray(R_DIAG, np.float64))
    Rx = np.outer(sq, sq) * Cr / np.outer(dr, dr)
    Rx = 0.5 * (Rx + Rx.T)
    leg = np.arange(12) // 3
    Rb = np.where(leg[:, None] == leg[None, :], Rx, 0.0)   # its leg blocks only
    Q = np.diag(Q_DIAG)
    for N in [int(v) for v in sys.argv[1:]] or [16, 20, 24]:
        B = 12
        bt = make_batch(B, N, seed=70 + N, gaits=("trot10", "pace10", "bound8"), robots=("a1", "aliengo"))
        bt["contact"][:] = 1.0   # standing: the interior-point class
        bt["contact"][1::3, N // 2:, 2] = 0.0
        for name, R in (("cross-leg R", Rx), ("leg-block R", Rb)):
            eng = LinearMpc(horizon=N, robot="a1", Q=Q, R=R)
            res = eng.solve(bt["x0"], bt["xref"], bt["contact"], bt["feet"], robot=bt["robot"], return_all=True)
            torch.cuda.synchronize()
            u0, U = res.u0.cpu().numpy(), res.U.cpu().numpy().reshape(B, -1)
            st, it = res.status.cpu().numpy(), res.iterations.cpu().numpy()
            errs = []
            for b in range(B):
                x, _, _ = oracle_solution(bt, b, N, Q=Q, R=R)
                errs.append(max(rel_err_u0(u0[b], x[:12]), rel_err_u0(U[b], x)))
            # one standing robot alone (latency), warm caches, cold solve
            one = {k: v[:1] for k, v in bt.items()}
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                eng.solve(one["x0"], one["xref"], one["contact"], one["feet"], robot=one["robot"])
            torch.cuda.synchronize()
            ev0.record()
            for _ in range(10):
                eng.solve(one["x0"], one["xref"], one["contact"], one["feet"], robot=one["robot"])
            ev1.record()
            torch.cuda.synchronize()
            ev2, ev3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev2.record()
            for _ in range(5):
                eng.solve(bt["x0"], bt["xref"], bt["contact"], bt["feet"], robot=bt["robot"])
            ev3.record()
            torch.cuda.synchronize()
            print(f"N={N} {name}: status {np.bincount(st, minlength=6).tolist()} worst rel err {max(errs):.2e} "
                  f"median {np.median(errs):.2e}; factorisations {it.tolist()}; robot 0 alone "
                  f"{ev0.elapsed_time(ev1) / 10:.3f} ms, the 12 robots {ev2.elapsed_time(ev3) / 5:.3f} ms per solve")


if __name__ == "__main__":
    main()
