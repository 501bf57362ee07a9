"""GPU diagnostic for the interior-point class: runs golden standing cases through a
-DMPCQP_IPM_DEBUG build (tools/libmpcqp_ipmdbg.so, built by `python tools/ipm_debug.py
build` on the CPU) and prints the per-iteration trace next to the release build's error."""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pympc-quadruped_amd"), os.path.join(ROOT, "tests")]
DBG = os.environ.get("IPM_DBG_LIB", os.path.join(ROOT, "tools", "libmpcqp_ipmdbg.so"))

if len(sys.argv) > 1 and sys.argv[1] == "build":
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-DMPCQP_IPM_DEBUG", "-I" + os.path.join(ROOT, "include"), "-o", DBG,
                    os.path.join(ROOT, "pympc-quadruped_amd", "csrc", "mpcqp.hip")], check=True)
    sys.exit(0)

import torch  # noqa: E402
from mpcqp import _lib  # noqa: E402
from helpers import rel_err_u0  # noqa: E402

N = int(os.environ.get("N", "16"))
cases = [int(c) for c in os.environ.get("CASES", "5,6,15").split(",")]
FLEET = int(os.environ.get("FLEET", "0"))   # > 0: that many robots (the cases repeated), mean cycles only
z = np.load(os.path.join(ROOT, "tests", "golden", f"formulation_N{N}.npz"), allow_pickle=False)
bt = {k: z[k][cases] for k in ("x0", "xref", "contact", "feet", "robot")}
if FLEET:
    bt = {k: np.concatenate([v] * (FLEET // len(cases) + 1))[:FLEET] for k, v in bt.items()}
# debug build: same call through the diagnostic library
lib = ctypes.CDLL(DBG)
params = _lib.MpcqpParams()
lib.mpcqp_default_params.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.mpcqp_default_params(ctypes.byref(params), N)
ctx = ctypes.c_void_p()
lib.mpcqp_create.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
assert lib.mpcqp_create(ctypes.byref(params), 0, ctypes.byref(ctx)) == 0
dev = torch.device("cuda:0")
t = {k: torch.as_tensor(np.ascontiguousarray(v, dtype=np.float32)).to(dev) for k, v in bt.items()}
B = len(cases)
u0d = torch.empty((B, 12), device=dev)
Ud = torch.zeros((B, N * 12), device=dev)
st = torch.empty((B,), dtype=torch.int32, device=dev)
itd = torch.empty((B,), dtype=torch.int32, device=dev)
p = lambda x: ctypes.c_void_p(x.data_ptr())
lib.mpcqp_solve.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 10
rc = lib.mpcqp_solve(ctx, B, p(t["x0"]), p(t["xref"]), p(t["contact"]), p(t["feet"]), p(t["robot"]), p(u0d),
                     p(Ud), p(st), p(itd), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
assert rc == 0, rc
D = Ud.cpu().numpy()
if FLEET:
    cyc = D[:, N * 12 - 8:].astype(np.float64)
    print(f"fleet of {FLEET} ({len(cases)} cases repeated): mean cycles per robot: gradient {cyc[:, 0].mean():.3g} "
          f"factor {cyc[:, 1].mean():.3g} lsolve {cyc[:, 2].mean():.3g} total {cyc[:, 3].mean():.3g}; factor T "
          f"{cyc[:, 4].mean():.3g} GJ {cyc[:, 5].mean():.3g} S store {cyc[:, 6].mean():.3g} sym {cyc[:, 7].mean():.3g}; "
          f"factorisations mean {itd.cpu().numpy().mean():.2f}")
    sys.exit(0)
for i, c in enumerate(cases):
    print(f"--- case {c} trace (it, mu, polish stat/g, slack min, lam min, nfact, gscale, hscale)")
    cyc = D[i][N * 12 - 8:]
    print(f"    cycles: gradient {cyc[0]:.3g} factor {cyc[1]:.3g} lsolve {cyc[2]:.3g} total {cyc[3]:.3g}; "
          f"factor T {cyc[4]:.3g} GJ {cyc[5]:.3g} S store {cyc[6]:.3g} sym {cyc[7]:.3g}")
    tr = D[i][:(N * 12 - 8) // 8 * 8].reshape(-1, 8)
    for row in tr:
        if row[0] == 0:
            break
        print("  " + " ".join(f"{v:10.3e}" for v in row))
lib.mpcqp_destroy.argtypes = [ctypes.c_void_p]
lib.mpcqp_destroy(ctx)
