"""CPU: the interior-point class's per-foot-step algebra (csrc/mpcqp_ipm_foot.h),
compiled for the host with g++ -- the multiplier check that decides whether a
polished active set is the optimum (g in the cone of the foot's active rows)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pympc-quadruped_amd", "csrc")

SHIM = r'''
#include "mpcqp_ipm_foot.h"
extern "C" void cone_mult(const double* rows, int am, int nq, const double* g, double tol, double* best, int* drop) {
  double rw[6][3], gg[3] = {g[0], g[1], g[2]};
  for (int r = 0; r < 6; ++r) for (int x = 0; x < 3; ++x) rw[r][x] = rows[3 * r + x];
  ipm_cone_multipliers(rw, am, nq, gg, tol, *best, *drop);
}
extern "C" void inverse3(const double* a, double* o) {
  double aa[9], oo[9];
  for (int i = 0; i < 9; ++i) aa[i] = a[i];
  inv3(aa, oo);
  for (int i = 0; i < 9; ++i) o[i] = oo[i];
}
'''


@pytest.fixture(scope="module")
def foot(tmp_path_factory):
    d = tmp_path_factory.mktemp("foot")
    src, so = d / "shim.cpp", d / "libfoot.so"
    src.write_text(SHIM)
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-I", CSRC, "-o", str(so), str(src)], check=True)
    lib = ctypes.CDLL(str(so))
    dp = ctypes.POINTER(ctypes.c_double)
    lib.cone_mult.argtypes = [dp, ctypes.c_int, ctypes.c_int, dp, ctypes.c_double, dp, ctypes.POINTER(ctypes.c_int)]
    lib.inverse3.argtypes = [dp, dp]

    def mult(rows, am, nq, g, tol=1e-9):
        rows = np.ascontiguousarray(rows, np.float64)
        g = np.ascontiguousarray(g, np.float64)
        best, drop = ctypes.c_double(), ctypes.c_int()
        lib.cone_mult(rows.ctypes.data_as(dp), am, nq, g.ctypes.data_as(dp), tol, ctypes.byref(best),
                      ctypes.byref(drop))
        return best.value, drop.value

    def inv(a):
        a = np.ascontiguousarray(a, np.float64).reshape(9)
        o = np.zeros(9)
        lib.inverse3(a.ctypes.data_as(dp), o.ctypes.data_as(dp))
        return o.reshape(3, 3)

    return mult, inv


def _rows(mu, normal=(0.0, 0.0, 1.0)):
    from oracle.formulation import cone_rows
    c = np.asarray(cone_rows(mu, normal), np.float64)
    return np.vstack([c, -c[4:5]])   # + the fz <= ub row (-n . f >= -ub)


def test_inverse3(foot):
    _, inv = foot
    rng = np.random.default_rng(0)
    for _ in range(20):
        m = rng.normal(size=(3, 3))
        a = m @ m.T + 0.1 * np.eye(3)
        np.testing.assert_allclose(inv(a) @ a, np.eye(3), atol=1e-10)


@pytest.mark.parametrize("mu,normal", [(0.7, (0, 0, 1)), (0.2, (0.1, -0.2, 1.0)), (1.5, (0.0, 0.25, 1.0))])
def test_cone_multipliers_match_nnls(foot, mu, normal):
    """Every active set of the six cone rows, random gradients in and out of the cone:
    best > 0 exactly when g is a non-negative combination of the active rows (scipy
    NNLS as the independent check), -inf when g is outside their span."""
    from scipy.optimize import nnls
    mult, _ = foot
    rows = _rows(mu, np.asarray(normal) / np.linalg.norm(normal))
    rng = np.random.default_rng(1)
    for am in range(1, 64):
        rs = [r for r in range(6) if (am >> r) & 1]
        if 4 in rs and 5 in rs:
            continue   # n.f >= 0 and n.f <= ub cannot both bind (ub > 0)
        A = rows[rs]
        nq = np.linalg.matrix_rank(A)
        for trial in range(6):
            if trial < 3:
                lam = rng.uniform(0.1, 2.0, size=len(rs))
                g = A.T @ lam
            else:
                g = A.T @ rng.normal(size=len(rs)) if trial < 5 else rng.normal(size=3)
            best, drop = mult(rows, am, nq, g)
            in_span = np.linalg.lstsq(A.T, g, rcond=None)[1]
            resid = np.abs(A.T @ np.linalg.lstsq(A.T, g, rcond=None)[0] - g).max()
            if resid > 1e-8:
                assert best == -np.inf, (am, trial)
                continue
            _, rn = nnls(A.T, g)
            in_cone = rn < 1e-8
            assert (best > -1e-9) == in_cone, (am, trial, best, rn)
            if not in_cone:
                assert drop in rs
