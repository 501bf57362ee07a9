"""Diagnostic: solve one seeded batch with the library named by MPCQP_LIB and save
u0 / iterations / status (compare two libraries with two runs):
  MPCQP_LIB=tools/libB.so python tools/lib_compare.py out.npz [B] [N] [gaits]
(LC_RANGE=lo,hi: promise the stance range, e.g. 64,64 for an all-standing N = 16 fleet;
LC_STAND=1: every robot standing)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pympc-quadruped_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    from mpcqp import LinearMpc
    from mpcqp.synthetic import make_batch
    out = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    gaits = tuple(sys.argv[4].split(",")) if len(sys.argv) > 4 else ("trot10",)
    bt = make_batch(B, N, seed=1000, gaits=gaits, robots=("a1",))
    if os.environ.get("LC_STAND"):
        bt["contact"][:] = 1.0
    eng = LinearMpc(horizon=N, robot="a1", device="cuda:0")
    if os.environ.get("LC_RANGE"):   # "lo,hi": the caller's stance range (e.g. an all-standing fleet)
        eng.set_stance_range(*[int(v) for v in os.environ["LC_RANGE"].split(",")])
    res = eng.solve(bt["x0"], bt["xref"], bt["contact"], bt["feet"], robot=bt["robot"], return_all=True)
    torch.cuda.synchronize()
    print("iterations histogram", np.bincount(res.iterations.cpu().numpy()).tolist())
    np.savez(out, u0=res.u0.cpu().numpy(), it=res.iterations.cpu().numpy(), st=res.status.cpu().numpy(),
             U=res.U.cpu().numpy())
    if len(sys.argv) > 5:
        ref = np.load(sys.argv[5])
        it0, it1 = ref["it"], res.iterations.cpu().numpy()
        du = np.abs(res.u0.cpu().numpy() - ref["u0"]).max(1) / np.maximum(np.abs(ref["u0"]).max(1), 1e-3)
        print("iterations ref mean %.2f max %d | this mean %.2f max %d | robots with more iterations %d" %
              (it0.mean(), it0.max(), it1.mean(), it1.max(), int((it1 > it0).sum())))
        worst = np.argsort(du)[-5:]
        print("u0 rel diff max %.2e; worst robots %s" % (du.max(), [(int(i), float(du[i]), int(it0[i]), int(it1[i])) for i in worst]))
        print("status ref", np.bincount(ref["st"]), "this", np.bincount(res.status.cpu().numpy()))


if __name__ == "__main__":
    main()
