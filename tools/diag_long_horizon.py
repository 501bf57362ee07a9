"""Diagnostic: one robot per call at a horizon beyond 20 (the interior-point class alone),
printing status / iterations / time, to find a slow or stuck case.
  python tools/diag_long_horizon.py N case   (case: standing | trot | sparse | flight)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pympc-quadruped_amd")]


def main():
    import torch
    from mpcqp import LinearMpc
    from mpcqp.synthetic import make_batch
    N, case = int(sys.argv[1]), sys.argv[2]
    bt = make_batch(1, N, seed=400 + N, gaits=("trot10",), robots=("a1",))
    if case == "standing":
        bt["contact"][0] = 1.0
    elif case == "sparse":
        bt["contact"][0] = (np.random.default_rng(1).random((N, 4)) < 0.2).astype(np.float32)
    elif case == "flight":
        bt["contact"][0] = 0.0
    eng = LinearMpc(horizon=N, robot="a1", device="cuda:0")
    t = time.time()
    res = eng.solve(bt["x0"], bt["xref"], bt["contact"], bt["feet"], robot=bt["robot"], return_all=True)
    torch.cuda.synchronize()
    print(N, case, "status", int(res.status[0]), "iters", int(res.iterations[0]), "%.3f s" % (time.time() - t),
          "u0", res.u0.cpu().numpy()[0, :3], flush=True)


if __name__ == "__main__":
    main()
