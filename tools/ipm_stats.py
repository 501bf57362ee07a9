"""GPU: statistics of the interior-point class on standing robots (release build):
factorisations per robot, status, parity sample, and the launch time for B robots."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pympc-quadruped_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
from mpcqp import LinearMpc  # noqa: E402
from mpcqp.synthetic import make_batch  # noqa: E402

for N, robots, tilt in ((16, ("a1",), 0.0), (20, ("a1", "aliengo"), 15.0)):
    B = int(os.environ.get("B", "256"))
    bt = make_batch(B, N, seed=7, gaits=("trot10",), robots=robots, tilt_deg=tilt)
    bt["contact"][:] = 1.0
    eng = LinearMpc(horizon=N, robot="a1")
    d = {k: torch.as_tensor(v).cuda() for k, v in bt.items()}
    for _ in range(2):
        res = eng.solve(d["x0"], d["xref"], d["contact"], d["feet"], robot=d["robot"], return_all=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        res = eng.solve(d["x0"], d["xref"], d["contact"], d["feet"], robot=d["robot"], return_all=True)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    it = res.iterations.cpu().numpy()
    st = res.status.cpu().numpy()
    print(f"N={N} B={B} standing: {ms:.3f} ms/solve, factorisations mean {it.mean():.1f} "
          f"p50 {np.median(it):.0f} p90 {np.percentile(it, 90):.0f} max {it.max()}, "
          f"status {np.unique(st, return_counts=True)}")
    if os.environ.get("PARITY"):
        from helpers import oracle_solution, rel_err_u0
        U = res.U.cpu().numpy().reshape(B, -1)
        worst = max(rel_err_u0(U[b], oracle_solution(bt, b, N)[0]) for b in range(0, B, max(1, B // 8)))
        print(f"   parity worst {worst:.2e}")
