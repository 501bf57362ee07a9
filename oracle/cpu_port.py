"""ctypes front of oracle/libmpc_cpu.so -- the compiled CPU restatement of the
reference's per-tick formulate + solve (oracle/cpu_mpc.cpp).  TEST INFRASTRUCTURE and
bench.py's cpu_baseline leg only; the product path never imports this module."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libmpc_cpu.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        lib = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        lib.mpc_cpu_solve_batch.restype = ctypes.c_int
        lib.mpc_cpu_solve_batch.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp, ctypes.c_double, vp, vp,
                                            vp, vp, vp, vp, ctypes.c_int]
        _lib = lib
    return _lib


def solve_batch(bt, N, dt=0.05, q=None, r=None, threads=1):
    """U [B, N*12] float64, iterations [B], formulation / solve thread-seconds."""
    from .formulation import Q_DIAG, R_DIAG
    lib = load()
    B = int(bt["x0"].shape[0])
    arrs = [np.ascontiguousarray(bt[k], dtype=np.float32) for k in ("x0", "xref", "contact", "feet", "robot")]
    q = np.ascontiguousarray(Q_DIAG if q is None else q, dtype=np.float64)
    r = np.ascontiguousarray(R_DIAG if r is None else r, dtype=np.float64)
    U = np.zeros((B, N * 12))
    it = np.zeros(B, dtype=np.int32)
    tf, ts = ctypes.c_double(), ctypes.c_double()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    lib.mpc_cpu_solve_batch(B, int(N), *[p(a) for a in arrs], float(dt), p(q), p(r), p(U), p(it),
                            ctypes.byref(tf), ctypes.byref(ts), int(threads))
    return U, it, tf.value, ts.value
