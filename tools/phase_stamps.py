"""Diagnostic: per-phase and per-section cycles of the dense classes (s_memtime stamps).

Uses a separately built libmpcqp_stamps.so (-DMPCQP_STAMPS, `python tools/phase_stamps.py build`)
whose kernels write, per robot, into the U buffer taken as 256 u64 slots (mpcqp_solve.h):
[0, 7) phase stamps, 7 / 8 chip-wide start / end (s_memrealtime, 100 MHz), [16, 24) each wave's
HW_ID, [32 + 24 w, 56 + 24 w) wave w's section accumulators (lane k: section k) and event
counters.  The shipped library executes no stamp.  Prints median / max cycles per phase and, per
wave, the active set's cycles per iteration by section.
  python tools/phase_stamps.py [B] [N] [gaits] [seed]
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pympc-quadruped_amd"))
STAMPS_LIB = os.path.join(ROOT, "pympc-quadruped_amd", "mpcqp", "libmpcqp_stamps.so")
SLOTS = 256          # kStampU64 (mpcqp.hip)
PHASES = ["inputs, model, Ya/Yb, g", "H tile", "sweep H^-1", "active set", "KKT check", "-"]
# section k runs from SEC(k) to the next SEC (mpcqp_solve.h); lanes 3, 4, 14, 15 are counters
SECTIONS = {0: "argmin p + a_p rows", 1: "combo + LDS store", 2: "zs = A z (LDS)", 5: "add: q, 1/s, loads, coefs",
            6: "drop: R_l, H R_l, R H R_l", 8: "pair candidate", 9: "barrier", 10: "pair-step test",
            11: "ratio test (loads, div, argmin)", 12: "t2, step, x/u/s", 13: "rank-1 FMAs (P, R)",
            16: "pair accept bookkeeping", 17: "pair W rank-2", 18: "pair R rank-2"}
COUNTERS = {3: "pair tests", 4: "fresh choices", 14: "drops", 15: "pair steps"}


def run_raw(B, N, gaits, seed, with_iters=False):
    """Run the stamps build once (3 launches) and return the stamp slots [B][256] (u64)."""
    import torch
    from mpcqp import _lib
    from mpcqp.synthetic import make_batch
    _lib.LIB_PATH = os.environ.get("MPCQP_STAMPS_LIB") or STAMPS_LIB
    lib = _lib.load()
    p = _lib.default_params(N)
    ctx = ctypes.c_void_p()
    _lib.check(None, lib.mpcqp_create(ctypes.byref(p), 0, ctypes.byref(ctx)), "create")
    bt = make_batch(B, N, seed=seed, gaits=gaits, robots=("a1",))
    dev = torch.device("cuda:0")
    d = {k: torch.as_tensor(v).to(dev).contiguous() for k, v in bt.items()}
    u0 = torch.empty((B, 12), device=dev)
    U = torch.zeros((B, 2 * SLOTS), device=dev)
    st = torch.empty((B,), dtype=torch.int32, device=dev)
    it = torch.empty((B,), dtype=torch.int32, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    for _ in range(3):
        lib.mpcqp_solve(ctx, B, P(d["x0"]), P(d["xref"]), P(d["contact"]), P(d["feet"]), P(d["robot"]),
                        P(u0), P(U), P(st), P(it), ctypes.c_void_p(0))
    torch.cuda.synchronize()
    slots = U.cpu().numpy().view(np.uint64).reshape(B, SLOTS).astype(np.int64)
    if with_iters:
        return slots, it.cpu().numpy()
    return slots


def wave_sections(slots, w):
    return slots[:, 32 + 24 * w:56 + 24 * w]


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-DMPCQP_STAMPS", "-I" + os.path.join(ROOT, "include"), "-o", STAMPS_LIB,
                        os.path.join(ROOT, "pympc-quadruped_amd", "csrc", "mpcqp.hip")], check=True)
        return
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    gaits = tuple(sys.argv[3].split(",")) if len(sys.argv) > 3 else ("trot10",)
    seed = int(sys.argv[4]) if len(sys.argv) > 4 else 1000
    slots, iters = run_raw(B, N, gaits, seed, with_iters=True)
    ts = slots[:, :7]
    dts = np.diff(ts, axis=1)
    print(f"B={B} N={N}  iterations mean {iters.mean():.1f} max {iters.max()}")
    for k, name in enumerate(PHASES):
        print(f"  {name:26s} median {np.median(dts[:, k]):9.0f}  max {dts[:, k].max():9.0f} cycles")
    tot = ts[:, 6] - ts[:, 0]
    print(f"  {'total':26s} median {np.median(tot):9.0f}  max {tot.max():9.0f}")
    rt = slots[:, 7:9]
    if rt[:, 0].min() > 0:   # start / end over the whole launch: dispatch ramp and tail
        t0 = (rt[:, 0] - rt[:, 0].min()) * 0.01
        t1 = (rt[:, 1] - rt[:, 0].min()) * 0.01
        print(f"  robot start (us after the first): median {np.median(t0):.2f} p90 {np.percentile(t0, 90):.2f} "
              f"max {t0.max():.2f}; end median {np.median(t1):.2f} p90 {np.percentile(t1, 90):.2f} max {t1.max():.2f}")
    sel = iters > 0
    gi = dts[:, 3]
    print(f"  active-set cycles / iteration: median {np.median(gi[sel] / iters[sel]):.0f}")
    nw = int(((slots[:, 16:24] != 0).sum(1)).max())   # waves per workgroup (HW_ID written by each)
    sec0 = wave_sections(slots, 0)
    for k, name in COUNTERS.items():
        v = sec0[:, k]
        print(f"  count {name:14s} mean {v[sel].mean():6.1f}  max {v.max():4d}")
    hw = slots[:, 16:16 + nw]
    simd = (hw >> 4) & 3
    print(f"  waves per robot {nw}; SIMD of each wave (robot 0): {simd[0].tolist()}")
    print("  iteration histogram:", np.histogram(iters, bins=[0, 10, 20, 30, 40, 50, 60, 80, 200])[0].tolist())
    tot_it = iters[sel].sum()
    print("  cycles per iteration by section (batch mean), waves " + " / ".join(str(w) for w in range(nw)))
    for k, name in SECTIONS.items():
        vals = [wave_sections(slots, w)[sel, k].sum() / tot_it for w in range(nw)]
        print(f"    sec {k:2d} {name:32s} " + " ".join(f"{v:7.0f}" for v in vals))
    for i in np.argsort(tot)[-4:]:
        print(f"  slow robot {i}: total {tot[i]} iterations {iters[i]} phases {dts[i, :5].tolist()} "
              + " ".join(f"{COUNTERS[k]} {int(sec0[i, k])}" for k in COUNTERS))
        print("     wave 0 sections:", {SECTIONS[k]: int(sec0[i, k]) for k in SECTIONS})
        if nw > 1:
            print("     wave 1 sections:", {SECTIONS[k]: int(wave_sections(slots, 1)[i, k]) for k in SECTIONS})


if __name__ == "__main__":
    main()
