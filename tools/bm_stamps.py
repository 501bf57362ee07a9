"""Diagnostic: phase stamps and per-section cycles of the class-64 brain / muscle kernel
(csrc/mpcqp_bm.h) from a -DMPCQP_STAMPS build (tools/lib_bm_stamps.so); the shipped
library executes no stamp.
  python tools/bm_stamps.py [B] [N] [gaits]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pympc-quadruped_amd"))
from mpcqp import _lib  # noqa: E402
from mpcqp.synthetic import make_batch  # noqa: E402

PHASES = ["stage, model, g", "H build", "sweep (muscle) + x0", "brain init", "active set", "final x, KKT"]
BSEC = ["command (choose, corrections)", "wait A", "A->B: r, R update", "wait B", "B->A: decisions",
        "B->A: drop helper (y)"]
MSEC = ["(exit)", "wait A", "directions / H R_l", "wait B"]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    gaits = tuple(sys.argv[3].split(",")) if len(sys.argv) > 3 else ("trot10",)
    _lib.LIB_PATH = os.environ.get("MPCQP_STAMPS_LIB") or os.path.join(ROOT, "tools", "lib_bm_stamps.so")
    lib = _lib.load()
    p = _lib.default_params(N)
    ctx = ctypes.c_void_p()
    _lib.check(None, lib.mpcqp_create(ctypes.byref(p), 0, ctypes.byref(ctx)), "create")
    lib.mpcqp_set_stance_range(ctx, 0, 21)
    bt = make_batch(B, N, seed=1000, gaits=gaits, robots=("a1",))
    dev = torch.device("cuda:0")
    d = {k: torch.as_tensor(v).to(dev).contiguous() for k, v in bt.items()}
    u0 = torch.empty((B, 12), device=dev)
    U = torch.zeros((B, N, 12), device=dev)
    st = torch.empty((B,), dtype=torch.int32, device=dev)
    it = torch.empty((B,), dtype=torch.int32, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    for _ in range(3):
        lib.mpcqp_solve(ctx, B, P(d["x0"]), P(d["xref"]), P(d["contact"]), P(d["feet"]), P(d["robot"]),
                        P(u0), P(U), P(st), P(it), ctypes.c_void_p(0))
    torch.cuda.synchronize()
    raw = U.cpu().numpy().reshape(B, -1).view(np.uint64).astype(np.int64)
    ts = raw[:, :7]
    dts = np.diff(ts, axis=1)
    bs = raw[:, 8:24]
    ms = raw[:, 24:40]
    iters = it.cpu().numpy()
    passes, helpers = bs[:, 10], bs[:, 11]
    tot = ts[:, 6] - ts[:, 0]
    print(f"B={B} N={N} {'+'.join(gaits)}: iterations mean {iters.mean():.1f} max {iters.max()}, "
          f"passes mean {passes.mean():.1f} max {passes.max()}, drop helper rounds mean {helpers.mean():.2f} max {helpers.max()}")
    for k, name in enumerate(PHASES):
        print(f"  {name:28s} median {np.median(dts[:, k]):9.0f}  max {dts[:, k].max():9.0f} cycles")
    print(f"  {'total':28s} median {np.median(tot):9.0f}  max {tot.max():9.0f}")
    sel = passes > 0
    print(f"  active set cycles per round (passes + helper rounds): median "
          f"{np.median(dts[sel, 4] / (passes[sel] + helpers[sel])):.0f}")
    print("  brain sections, cycles per round (batch mean | slowest 8 robots mean):")
    slow = np.argsort(tot)[-8:]
    rounds = np.maximum(passes + helpers, 1)
    for k, name in enumerate(BSEC):
        print(f"    {name:32s} {np.mean(bs[sel, k] / rounds[sel]):8.0f} | {np.mean(bs[slow, k] / rounds[slow]):8.0f}")
    print("  muscle sections, cycles per round:")
    for k, name in enumerate(MSEC):
        print(f"    {name:32s} {np.mean(ms[sel, k] / rounds[sel]):8.0f} | {np.mean(ms[slow, k] / rounds[slow]):8.0f}")
    for i in slow[-4:]:
        print(f"  slow robot {i}: total {tot[i]} iterations {iters[i]} passes {passes[i]} helpers {helpers[i]} "
              f"phases {dts[i, :6].tolist()}")


if __name__ == "__main__":
    main()
