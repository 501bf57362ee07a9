"""Diagnostic: NumPy model of the brain / muscle split of the class-64 active set
(csrc/mpcqp_bm.h): the muscle wave holds P (reduced inverse Hessian) and x, the
brain wave holds R (multiplier map), s, u and every decision; each side applies the
previous step's rank update one pass late, and the step directions of a pass are
formed from the lagging matrices plus a correction for that pending update.  Checks
that the lagged bookkeeping reproduces the eager loop (tools/gi_sim.py, pair steps,
current-metric row keys): same passes, same optimum.
Usage: python tools/bm_sim.py [B] [N]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "pympc-quadruped_amd"))
from gi_sim import robot_qp, simulate  # noqa: E402
from mpcqp.synthetic import make_batch  # noqa: E402


def bm_solve(H, g, A, b, foot, tol=1e-9, max_iter=1000, eager=False):
    n = H.shape[0]
    m = A.shape[0]
    W = np.linalg.inv(H)
    # ---- muscle state
    P = W.copy()
    x = -W @ g
    # ---- brain state
    R = np.zeros((n, n))       # slot rows (lagging like P)
    occ = np.zeros(n, bool)
    u = np.zeros(n)
    s = A @ x - b
    wscale = np.max(np.diag(W))
    qm = np.einsum("ij,jk,ik->i", A, W, A)
    qfloor = max(1e-9 * wscale, 1e-30)
    pu = None   # pending update: dict(kind, ...) -- applied by both sides one pass late
    zs_prev = zs2_prev = None
    p = -1
    it = passes = drops = 0
    sp = up = 0.0

    def corr_coefs(a_row):
        """Correction coefficients of the pending update for a step direction of row a."""
        if pu is None:
            return None
        if pu["kind"] == "add":
            return (zs_prev_row(a_row) / pu["sigma"],)
        if pu["kind"] == "pair":
            v = np.array([zs_prev_row(a_row), zs2_prev_row(a_row)])
            return tuple(pu["Si"] @ v)
        return ((pu["Rl"] @ A[a_row]) / pu["eta"],)   # drop

    def zs_prev_row(c):
        return zs_prev[c]

    def zs2_prev_row(c):
        return zs2_prev[c]

    def muscle_dir(c, cf):
        z = P @ A[c]
        if pu is None:
            return z
        if pu["kind"] == "add":
            return z - cf[0] * pu["z"]
        if pu["kind"] == "pair":
            return z - cf[0] * pu["z"] - cf[1] * pu["z2"]
        return z + cf[0] * pu["Rl"]

    def brain_dir(c, cf):
        r = R @ A[c]
        if pu is None:
            return r
        if pu["kind"] == "add":
            e = np.zeros(n); e[pu["q"]] = 1.0
            return r - cf[0] * (pu["r"] - e)
        if pu["kind"] == "pair":
            ea = np.zeros(n); ea[pu["qa"]] = 1.0
            eb = np.zeros(n); eb[pu["qb"]] = 1.0
            return r - cf[0] * (pu["r"] - ea) - cf[1] * (pu["r2"] - eb)
        rr = r - cf[0] * pu["y"]
        rr[pu["l"]] = 0.0
        return rr

    def apply_pending():
        nonlocal P, R, x
        if pu is None:
            return
        if pu["kind"] == "add":
            e = np.zeros(n); e[pu["q"]] = 1.0
            P = P - np.outer(pu["z"], pu["z"]) / pu["sigma"]
            R = R - np.outer(pu["r"] - e, pu["z"]) / pu["sigma"]
            x = x + pu["t"] * pu["z"]
        elif pu["kind"] == "pair":
            ea = np.zeros(n); ea[pu["qa"]] = 1.0
            eb = np.zeros(n); eb[pu["qb"]] = 1.0
            Z = np.stack([pu["z"], pu["z2"]], 1)
            Rk = np.stack([pu["r"] - ea, pu["r2"] - eb], 1)
            P = P - Z @ pu["Si"] @ Z.T
            R = R - Rk @ pu["Si"] @ Z.T
            x = x + pu["tp"] * pu["z"] + pu["tq"] * pu["z2"]
        else:
            P = P + np.outer(pu["Rl"], pu["Rl"]) / pu["eta"]
            R = R - np.outer(pu["y"], pu["Rl"]) / pu["eta"]
            R[pu["l"]] = 0.0
            x = x + pu["t"] * pu["z"]

    while True:
        if eager and pu is not None:
            apply_pending()
            pu = None
        p2 = -1
        if p < 0:
            key = np.where(s < -tol, s / np.sqrt(np.maximum(qm, qfloor)), np.inf)
            if not np.isfinite(key.min()):
                break
            p = int(np.argmin(key))
            k2 = np.where(foot == foot[p], np.inf, key)
            p2 = int(np.argmin(k2)) if np.isfinite(k2.min()) else -1
            sp = s[p]
            up = 0.0
        it += 1
        passes += 1
        if it > max_iter:
            return None
        # barrier A: the command carries the pending update's correction coefficients
        cf = corr_coefs(p)
        cf2 = corr_coefs(p2) if p2 >= 0 else None
        z = muscle_dir(p, cf)
        r = brain_dir(p, cf)
        z2 = muscle_dir(p2, cf2) if p2 >= 0 else None
        r2 = brain_dir(p2, cf2) if p2 >= 0 else None
        # both sides now apply the pending update (B: R in the A->B window, M: P, x after B)
        apply_pending()
        pu = None
        zs = A @ z
        zsp = zs[p]
        thr = 1e-12 * (A[p] @ A[p]) * wscale
        if p2 >= 0:
            zs2 = A @ z2
            s12, s22 = zs2[p], zs2[p2]
            thr2 = 1e-12 * (A[p2] @ A[p2]) * wscale
            det = zsp * s22 - s12 * s12
            ok = zsp > thr and s22 > thr2 and det > thr2 * zsp
            if ok:
                sp2 = s[p2]
                tp = (s12 * sp2 - s22 * sp) / det
                tq = (s12 * sp - zsp * sp2) / det
                ok = tp > 0 and tq > 0 and not np.any(occ & (u - tp * r - tq * r2 < 0))
            if ok:
                u = np.where(occ, u - tp * r - tq * r2, u)
                s = s + tp * zs + tq * zs2
                s[p] = s[p2] = 0.0
                free = np.flatnonzero(~occ)
                qa, qb = int(free[0]), int(free[1])
                u[qa], u[qb] = tp, tq
                occ[qa] = occ[qb] = True
                Si = np.array([[s22, -s12], [-s12, zsp]]) / det
                ZS = np.stack([zs, zs2], 1)
                qm = qm - np.einsum("ij,jk,ik->i", ZS, Si, ZS)
                pu = dict(kind="pair", Si=Si, z=z, z2=z2, r=r, r2=r2, qa=qa, qb=qb, tp=tp, tq=tq)
                zs_prev, zs2_prev = zs, zs2
                p = -1
                it += 1
                continue
        ratios = np.where(occ & (r > 0), u / np.where(r > 0, r, 1), np.inf)
        l = int(np.argmin(ratios))
        t1 = ratios[l]
        t2 = -sp / zsp if zsp > thr else np.inf
        t = min(t1, t2)
        if not np.isfinite(t):
            return None
        u = np.where(occ, u - t * r, u)
        s = s + t * zs
        sp = sp + t * zsp
        up += t
        if t2 <= t1:
            q = int(np.flatnonzero(~occ)[0])
            u[q] = up
            occ[q] = True
            s[p] = 0.0
            qm = qm - zs * zs / zsp
            pu = dict(kind="add", sigma=zsp, q=q, z=z, r=r, t=t)
            zs_prev = zs
            p = -1
        else:
            # helper round: the muscle forms t = H R_l (H's copy), the brain y = R t
            Rl = R[l].copy()
            y = R @ (H @ Rl)
            eta = y[l]
            qm = qm + (A @ Rl) ** 2 / eta
            u[l] = 0.0
            occ[l] = False
            # the row that left the active set
            drops += 1
            pu = dict(kind="drop", eta=eta, Rl=Rl, y=y, l=l, z=z, t=t)
    apply_pending()
    return dict(x=x, passes=passes, it=it, drops=drops)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    bt = make_batch(B, N, seed=1000, gaits=("trot10",), robots=("a1",))
    worst = 0.0
    for bb in range(B):
        H, g, A, b, foot = robot_qp(bt, bb, N)
        ref = bm_solve(H, g, A, b, foot, eager=True)
        got = bm_solve(H, g, A, b, foot)
        err = np.abs(got["x"] - ref["x"]).max() / max(np.abs(ref["x"]).max(), 1e-3)
        worst = max(worst, err)
        if got["passes"] != ref["passes"]:
            print("robot", bb, "passes", got["passes"], "eager", ref["passes"])
    print("worst rel x difference vs the eager loop: %.2e" % worst)


if __name__ == "__main__":
    main()
