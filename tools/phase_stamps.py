"""Diagnostic: per-phase cycle shares of the engine kernel (s_memtime stamps).

Uses a separately built libmpcqp_stamps.so (-DMPCQP_STAMPS) whose kernel writes
7 timestamps per robot into the U buffer; the shipped library executes no stamp.
Prints median / max cycles per phase over the batch.
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pympc-quadruped_amd"))
from mpcqp import _lib  # noqa: E402
from mpcqp.synthetic import make_batch  # noqa: E402

PHASES = ["inputs, model, Ya/Yb, g", "H tile", "sweep H^-1", "active set", "KKT check", "-"]


def run_raw(B, N, gaits, seed, with_iters=False):
    """Run the stamps build once (3 launches) and return U as a NumPy array."""
    _lib.LIB_PATH = os.environ.get("MPCQP_STAMPS_LIB") or os.path.join(ROOT, "pympc-quadruped_amd", "mpcqp",
                                                                       "libmpcqp_stamps.so")
    lib = _lib.load()
    p = _lib.default_params(N)
    ctx = ctypes.c_void_p()
    _lib.check(None, lib.mpcqp_create(ctypes.byref(p), 0, ctypes.byref(ctx)), "create")
    bt = make_batch(B, N, seed=seed, gaits=gaits, robots=("a1",))
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
    if with_iters:
        return U.cpu().numpy(), it.cpu().numpy()
    return U.cpu().numpy()


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    gaits = tuple(sys.argv[3].split(",")) if len(sys.argv) > 3 else ("trot10",)
    seed = int(sys.argv[4]) if len(sys.argv) > 4 else 1000
    Un, iters = run_raw(B, N, gaits, seed, with_iters=True)
    ts = Un.reshape(B, -1).view(np.uint64)[:, :7].astype(np.int64)
    dts = np.diff(ts, axis=1)
    print(f"B={B} N={N}  iterations mean {iters.mean():.1f} max {iters.max()}")
    for k, name in enumerate(PHASES):
        print(f"  {name:26s} median {np.median(dts[:, k]):9.0f}  max {dts[:, k].max():9.0f} cycles")
    tot = ts[:, 6] - ts[:, 0]
    print(f"  {'total':26s} median {np.median(tot):9.0f}  max {tot.max():9.0f}")
    # start / end over the whole launch (s_memrealtime: 100 MHz, chip-wide): dispatch ramp and tail
    rt = Un.reshape(B, -1).view(np.uint64)[:, 44:46].astype(np.int64)
    if rt[:, 0].min() > 0:
        t0 = (rt[:, 0] - rt[:, 0].min()) * 0.01
        t1 = (rt[:, 1] - rt[:, 0].min()) * 0.01
        print(f"  robot start (us after the first): median {np.median(t0):.2f} p90 {np.percentile(t0, 90):.2f} "
              f"max {t0.max():.2f}; end median {np.median(t1):.2f} p90 {np.percentile(t1, 90):.2f} max {t1.max():.2f}")
    for i in np.argsort(tot)[-4:]:
        print(f"  slow robot {i}: total {tot[i]} iterations {iters[i]} phases {dts[i, :5].tolist()}")
    gi = dts[:, 3]
    sel = iters > 0
    print(f"  active-set cycles / iteration: median {np.median(gi[sel] / iters[sel]):.0f}")
    sec = Un.reshape(B, -1).view(np.uint64)[:, 8:24].astype(np.int64)
    sec1 = Un.reshape(B, -1).view(np.uint64)[:, 26:42].astype(np.int64)
    # section k runs from SEC(k) to the next SEC (mpcqp_solve.h)
    names = ["argmin p + a_p rows", "combo + LDS store", "zs = A z (LDS)", "-", "-", "add: q, 1/s, loads, coefs",
             "drop: R_l, H R_l, R H R_l", "-", "pair candidate", "barrier", "pair-step test",
             "ratio test (loads, div, argmin)", "t2, step, x/u/s", "rank-1 FMAs (P, R)", "-", "-"]
    # event counters (slots 3, 4, 14, 15): pair tests, fresh row choices, drops, pair steps
    cnt = {"pair tests": sec[:, 3], "fresh choices": sec[:, 4], "drops": sec[:, 14], "pair steps": sec[:, 15]}
    for k, v in cnt.items():
        print(f"  count {k:14s} mean {v[sel].mean():6.1f}  max {v.max():4d}")
    hw = Un.reshape(B, -1).view(np.uint64)[:, 24:26].astype(np.int64)
    simd = (hw >> 4) & 3
    cu = ((hw >> 8) & 15) | (((hw >> 13) & 7) << 4)
    print(f"  waves 0/1 on the same SIMD: {(simd[:, 0] == simd[:, 1]).mean():.3f}  same CU: "
          f"{(cu[:, 0] == cu[:, 1]).mean():.3f}  raw {hw[:2].tolist()}")
    print("  iteration histogram:", np.histogram(iters, bins=[0, 10, 20, 30, 40, 50, 60, 80, 200])[0].tolist())
    for i in np.argsort(tot)[-6:]:
        print(f"  robot {i}: it {iters[i]} fresh {sec[i, 4]} pair tests {sec[i, 3]} pairs {sec[i, 15]} "
              f"drops {sec[i, 14]} loop cycles {dts[i, 3]} per pass {dts[i, 3] / max(1, iters[i] - sec[i, 15]):.0f}")
        print("     sections:", {names[k]: int(sec[i, k]) for k in range(16) if names[k] != "-"})
        ex = Un.reshape(B, -1).view(np.uint64)[i, 46:52].astype(np.int64)
        if ex.any():
            print("     pair step split (wave 0 / wave 1): decision (sec 10)", int(sec[i, 10]), int(sec1[i, 10]),
                  "| accept bookkeeping", int(ex[0]), int(ex[3]), "| W rank-2", int(ex[1]), int(ex[4]),
                  "| R rank-2", int(ex[2]), int(ex[5]))
        print("     wave 1:  ", {names[k]: int(sec1[i, k]) for k in range(16) if names[k] != "-"})
    tot_it = iters[sel].sum()
    for k, name in enumerate(names):
        if name != "-":
            print(f"  sec {name:20s} cycles/iteration (batch mean) {sec[sel, k].sum() / tot_it:8.0f}"
                  f"   wave 1 {sec1[sel, k].sum() / tot_it:8.0f}")


if __name__ == "__main__":
    main()
