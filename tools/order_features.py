"""Diagnostic (round 5): per-robot iteration counts of the bench's seeded batches (GPU) next
to the inputs, for fitting the dispatch-order key of mpcqp_order_kernel offline.
  python tools/order_features.py out.npz config5 [k ...]   (k: the bench's batch index, seed 1000 (k + 1))"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pympc-quadruped_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import CONFIGS
    from mpcqp import LinearMpc
    from mpcqp.synthetic import make_batch
    out, cfg = sys.argv[1], sys.argv[2]
    ks = [int(a) for a in sys.argv[3:]] or [0, 1]
    B, N, gaits, robots, tilt = CONFIGS[cfg]
    eng = LinearMpc(horizon=N, robot="a1", device="cuda:0")
    rec = {}
    for k in ks:
        bt = make_batch(B, N, seed=1000 * (k + 1), gaits=gaits, robots=robots, tilt_deg=tilt)
        res = eng.solve(bt["x0"], bt["xref"], bt["contact"], bt["feet"], robot=bt["robot"], return_all=True)
        torch.cuda.synchronize()
        for key, v in bt.items():
            rec[f"{key}_{k}"] = v
        rec[f"it_{k}"] = res.iterations.cpu().numpy()
        rec[f"st_{k}"] = res.status.cpu().numpy()
    np.savez(out, **rec)
    print("saved", out, {k: v.shape for k, v in rec.items() if k.startswith("it")})


if __name__ == "__main__":
    main()
