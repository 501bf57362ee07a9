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
extern "C" void foot_weight(const double* rows, int live, const double* d, const double* rh, double* W) {
  double rw[6][3], dd[6], r9[9], w9[9];
  for (int r = 0; r < 6; ++r) { dd[r] = d[r]; for (int x = 0; x < 3; ++x) rw[r][x] = rows[3 * r + x]; }
  for (int i = 0; i < 9; ++i) r9[i] = rh[i];
  ipm_foot_weight(rw, live, dd, r9, w9);
  for (int i = 0; i < 9; ++i) W[i] = w9[i];
}
extern "C" int foot_nullspace(const double* rows, int am, double h5, const double* rh, double* pj, double* fp,
                              double* W) {
  double rw[6][3], r9[9], p9[9], f3[3], w9[9];
  for (int r = 0; r < 6; ++r) for (int x = 0; x < 3; ++x) rw[r][x] = rows[3 * r + x];
  for (int i = 0; i < 9; ++i) r9[i] = rh[i];
  const int nq = ipm_foot_nullspace(rw, am, h5, r9, p9, f3, w9);
  for (int i = 0; i < 9; ++i) { pj[i] = p9[i]; W[i] = w9[i]; }
  for (int i = 0; i < 3; ++i) fp[i] = f3[i];
  return nq;
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
    lib.foot_weight.argtypes = [dp, ctypes.c_int, dp, dp, dp]
    lib.foot_nullspace.argtypes = [dp, ctypes.c_int, ctypes.c_double, dp, dp, dp, dp]
    lib.foot_nullspace.restype = ctypes.c_int

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

    def c(a):
        return np.ascontiguousarray(a, np.float64)

    def weight(rows, live, d, rh):
        W = np.zeros(9)
        rows, d, rh = c(rows), c(d), c(rh).reshape(9)
        lib.foot_weight(rows.ctypes.data_as(dp), live, d.ctypes.data_as(dp), rh.ctypes.data_as(dp),
                        W.ctypes.data_as(dp))
        return W.reshape(3, 3)

    def nullspace(rows, am, h5, rh):
        pj, fp, W = np.zeros(9), np.zeros(3), np.zeros(9)
        rows, rh = c(rows), c(rh).reshape(9)
        nq = lib.foot_nullspace(rows.ctypes.data_as(dp), am, h5, rh.ctypes.data_as(dp), pj.ctypes.data_as(dp),
                                fp.ctypes.data_as(dp), W.ctypes.data_as(dp))
        return nq, pj.reshape(3, 3), fp, W.reshape(3, 3)

    lib.weight, lib.nullspace = weight, nullspace
    return mult, inv, lib


def _rows(mu, normal=(0.0, 0.0, 1.0)):
    from oracle.formulation import cone_rows
    c = np.asarray(cone_rows(mu, normal), np.float64)
    return np.vstack([c, -c[4:5]])   # + the fz <= ub row (-n . f >= -ub)


def test_inverse3(foot):
    _, inv, _ = foot
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
    mult, _, _ = foot
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


def _leg_block(rng):
    """A full symmetric positive-definite 3 x 3 leg block of R (mpcqp_set_weights)."""
    S = rng.normal(size=(3, 3))
    return 1e-5 * np.eye(3) + 1e-6 * (S @ S.T)


def test_foot_weight_full_leg_block(foot):
    """W = (R_leg + sum_live d_r a_r a_r^T)^-1 with a full (non-diagonal) 3 x 3 R block."""
    lib = foot[2]
    rng = np.random.default_rng(3)
    rows = _rows(0.6, np.array([0.1, 0.05, 1.0]) / np.linalg.norm([0.1, 0.05, 1.0]))
    for live in (0, 1, 0b10101, 0b111111, 0b011110):
        d = rng.uniform(0.0, 50.0, size=6)
        rh = _leg_block(rng)
        want = rh.copy()
        for r in range(6):
            if (live >> r) & 1:
                want += d[r] * np.outer(rows[r], rows[r])
        # cond(want) reaches ~1e7 (d_r / R): the adjugate inverse's forward error is ~cond x eps
        inv = np.linalg.inv(want)
        err = np.abs(lib.weight(rows, live, d, rh) - inv).max() / np.abs(inv).max()
        assert err < 100 * np.finfo(float).eps * np.linalg.cond(want), (live, err)


def test_foot_nullspace_full_leg_block(foot):
    """The polish's reduced stage problem with a full 3 x 3 R block: pj projects onto the
    null space of the active rows, fp is their minimum-norm solution (a_5 . fp = h5),
    and W = pj (pj R pj + I - pj)^-1 pj, i.e. the inverse of R restricted to the null
    space."""
    lib = foot[2]
    rng = np.random.default_rng(4)
    rows = _rows(0.7)
    for am in (0, 1, 0b100000, 0b100001, 0b000011, 0b001101):
        rh = _leg_block(rng)
        h5 = -120.0
        nq, pj, fp, W = lib.nullspace(rows, am, h5, rh)
        A = rows[[r for r in range(6) if (am >> r) & 1]]
        assert nq == (np.linalg.matrix_rank(A) if len(A) else 0)
        want_pj = np.eye(3) - (np.linalg.pinv(A) @ A if len(A) else 0.0)
        np.testing.assert_allclose(pj, want_pj, atol=1e-12)
        h = np.array([h5 if r == 5 else 0.0 for r in range(6) if (am >> r) & 1])
        np.testing.assert_allclose(fp, np.linalg.pinv(A) @ h if len(A) else np.zeros(3), atol=1e-9)
        want_W = pj @ np.linalg.inv(pj @ rh @ pj + np.eye(3) - pj) @ pj
        np.testing.assert_allclose(W, want_W, rtol=1e-8, atol=1e-6 * np.abs(want_W).max())
