"""Diagnostic: per-tile-column sweep timestamps of the large class (stamps build)."""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pympc-quadruped_amd"))
from mpcqp import _lib  # noqa: E402
from mpcqp.synthetic import make_batch  # noqa: E402

B, N = int(sys.argv[1]), int(sys.argv[2])
_lib.LIB_PATH = os.path.join(ROOT, "pympc-quadruped_amd", "mpcqp", "libmpcqp_stamps.so")
lib = _lib.load()
p = _lib.default_params(N)
ctx = ctypes.c_void_p()
_lib.check(None, lib.mpcqp_create(ctypes.byref(p), 0, ctypes.byref(ctx)), "create")
bt = make_batch(B, N, seed=1000, gaits=("trot10", "pace10", "bound8"), robots=("a1",))
dev = torch.device("cuda:0")
d = {k: torch.as_tensor(v).to(dev).contiguous() for k, v in bt.items()}
u0 = torch.empty((B, 12), device=dev)
U = torch.zeros((B, N, 12), device=dev)
st = torch.empty((B,), dtype=torch.int32, device=dev)
it = torch.empty((B,), dtype=torch.int32, device=dev)
P = lambda t: ctypes.c_void_p(t.data_ptr())
for _ in range(2):
    lib.mpcqp_solve(ctx, B, P(d["x0"]), P(d["xref"]), P(d["contact"]), P(d["feet"]), P(d["robot"]),
                    P(u0), P(U), P(st), P(it), ctypes.c_void_p(0))
torch.cuda.synchronize()
ts = U.cpu().numpy().reshape(B, -1).view(np.uint64).astype(np.int64)
sw = ts[:, 8:8 + 16]
print("sweep start-of-tile-column deltas (median over robots):", np.median(np.diff(sw[:, :12], axis=1), axis=0))
print("phase stamps deltas:", np.median(np.diff(ts[:, :7], axis=1), axis=0))
