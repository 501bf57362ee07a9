"""Diagnostic: CPU simulation of the engine's projected Goldfarb-Idnani loop
(mpcqp_solve.h) with k-row "multi-add" steps, to count loop passes per robot.

Policy k = 1: single steps only; k = 2: the engine's pair steps; k > 2: up to k
rows from distinct foot-steps added at once when the equality-constrained step
keeps every multiplier positive (nested fallback to fewer rows, then a single
GI step).  Decisions follow the engine: the most violated row in the dual metric
(scaled by the initial W), partner rows the best of other foot-steps.
Usage: python tools/gi_sim.py [B] [k ...]   (GI_METRIC=W: rows keyed in the initial metric;
GI_N / GI_GAITS: horizon and gait mix, default 10 / trot10)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pympc-quadruped_amd"))
from oracle import formulation as F  # noqa: E402
from oracle import qp as Q  # noqa: E402
from mpcqp.synthetic import make_batch  # noqa: E402


def robot_qp(bt, b, N):
    x0 = bt["x0"][b]
    rec = bt["robot"][b]
    inertia = np.array([[rec[1], rec[2], rec[3]], [rec[2], rec[4], rec[5]], [rec[3], rec[5], rec[6]]],
                       dtype=np.float32)
    o = F.formulate(x0, bt["xref"][b].reshape(-1), bt["contact"][b].reshape(-1), bt["feet"][b].astype(np.float64),
                    inertia, float(rec[0]), N, mu=float(rec[7]), fz_max=float(rec[8]),
                    normal=rec[9:12].astype(np.float64))
    contact = bt["contact"][b].reshape(-1)
    idx = Q.swing_elimination(contact, N)
    H = o["H"][np.ix_(idx, idx)].astype(np.float64)
    g = o["g"][idx].astype(np.float64)
    nv = rec[9:12].astype(np.float64)
    nv = nv / np.linalg.norm(nv) if np.linalg.norm(nv) > 0 else np.array([0, 0, 1.0])
    t1 = np.array([1.0, 0, 0]) - nv[0] * nv
    t1 /= np.linalg.norm(t1)
    t2 = np.cross(nv, t1)
    mu, fz = float(rec[7]), float(rec[8])
    cone = [t1 + mu * nv, -t1 + mu * nv, t2 + mu * nv, -t2 + mu * nv, -nv]   # n.f >= 0 implied (mu > 0)
    S = len(idx) // 3
    ub = [float(contact[k]) * fz for k in range(len(contact)) if contact[k] > 0]
    A, bb, foot = [], [], []
    for j in range(S):
        for r, a in enumerate(cone):
            row = np.zeros(3 * S)
            row[3 * j:3 * j + 3] = a
            A.append(row)
            bb.append(-ub[j] if r == 4 else 0.0)
            foot.append(j)
    return H, g, np.array(A), np.array(bb), np.array(foot)


def simulate(H, g, A, b, foot, kmax, tol=1e-9, max_pass=2000, ratio=0.0, stop_after_drops=10**9, W0=None,
             metric="P", init_rows=None):
    n = H.shape[0]
    W = np.linalg.inv(H) if W0 is None else W0.copy()
    P = W.copy()
    R = np.zeros((n, n))          # slot rows
    occ = np.zeros(n, bool)
    slot_row = -np.ones(n, int)
    u = np.zeros(n)
    x = -W @ g
    if init_rows is not None and len(init_rows):
        # warm start: the equality-constrained optimum on init_rows (a valid dual
        # active-set iterate when every multiplier is >= 0)
        G = list(init_rows)
        k = len(G)
        AG = A[G]
        M = AG @ W @ AG.T
        Mi = np.linalg.pinv(M)
        lam = Mi @ (b[G] - AG @ x)
        x = x + W @ AG.T @ lam
        P = W - W @ AG.T @ Mi @ AG @ W
        R[:k] = Mi @ AG @ W
        occ[:k] = True
        slot_row[:k] = G
        u[:k] = lam
    rn = 1.0 / np.sqrt(np.einsum("ij,jk,ik->i", A, W, A))
    wscale = np.max(np.diag(W))
    passes = it = drops = multi = 0
    cost = 0.0   # crude per-pass cost model (single-add pass = 1)
    p = -1
    up = 0.0
    while passes < max_pass:
        s = A @ x - b
        s[slot_row[occ]] = np.inf        # active rows
        if p < 0:
            if metric == "P":   # the kernel's rule: current metric a P a (steepest dual ascent)
                scale = 1.0 / np.sqrt(np.maximum(np.einsum("ij,jk,ik->i", A, P, A), 1e-9 * wscale))
            else:               # round-1/2 rule: initial metric a W a
                scale = rn
            key = np.where(s < -tol, s * scale, np.inf)
            if not np.isfinite(key.min()):
                break
            cands = []
            used = set()
            order = np.argsort(key, kind="stable")
            klim = kmax if drops < stop_after_drops else 1
            for c in order:
                if not np.isfinite(key[c]) or len(cands) >= klim:
                    break
                if foot[c] in used:
                    continue
                if cands and key[c] > ratio * key[cands[0]]:   # partners at least `ratio` as violated
                    break
                cands.append(c)
                used.add(foot[c])
            p = cands[0]
            up = 0.0
        else:
            cands = [p]
        passes += 1
        # multi-add test, nested
        done = False
        cost += 1.0 + 0.35 * (len(cands) - 1)   # base pass + per extra candidate (argmin, combo, zs)
        if len(cands) > 1:
            Z = P @ A[cands].T
            Rk = R @ A[cands].T
            Sm = A[cands] @ Z
            for k in range(len(cands), 1, -1):
                Sk = Sm[:k, :k]
                thrk = 1e-12 * (A[cands[:k]] ** 2).sum(1) * wscale
                if np.any(np.diag(Sk) <= thrk):
                    continue
                try:
                    t = -np.linalg.solve(Sk, s[cands[:k]])
                except np.linalg.LinAlgError:
                    continue
                if np.any(t <= 0):
                    continue
                unew = u - Rk[:, :k] @ t
                if np.any(unew[occ] < 0):
                    continue
                # accept k rows
                x = x + Z[:, :k] @ t
                u = np.where(occ, unew, u)
                free = np.flatnonzero(~occ)[:k]
                E = np.zeros((n, k))
                E[free, np.arange(k)] = 1.0
                Si = np.linalg.inv(Sk)
                P = P - Z[:, :k] @ Si @ Z[:, :k].T
                R = R - (Rk[:, :k] - E) @ Si @ Z[:, :k].T
                for j, q in enumerate(free):
                    occ[q] = True
                    slot_row[q] = cands[j]
                    u[q] = t[j]
                it += k
                multi += k > 1
                cost += 0.2 * k   # rank-k update beyond the rank-1 of a single add
                p = -1
                done = True
                break
        if done:
            continue
        it += 1
        z = P @ A[p]
        r = R @ A[p]
        zsp = A[p] @ z
        sp = A[p] @ x - b[p]
        thr = 1e-12 * (A[p] ** 2).sum() * wscale
        ratios = np.where(occ & (r > 0), u / np.where(r > 0, r, 1), np.inf)
        l = int(np.argmin(ratios))
        t1 = ratios[l]
        t2 = -sp / zsp if zsp > thr else np.inf
        tstep = min(t1, t2)
        if not np.isfinite(tstep):
            return dict(passes=passes, it=it, drops=drops, multi=multi, status="infeasible")
        if np.isfinite(t2):
            x = x + tstep * z
        u = np.where(occ, u - tstep * r, u)
        up += tstep
        if t2 <= t1:
            q = int(np.flatnonzero(~occ)[0])
            e = np.zeros(n)
            e[q] = 1.0
            P = P - np.outer(z, z) / zsp
            R = R - np.outer(r - e, z) / zsp
            occ[q] = True
            slot_row[q] = p
            u[q] = up
            p = -1
        else:
            Rl = R[l].copy()
            y = R @ (H @ Rl)
            eta = y[l]
            P = P + np.outer(Rl, Rl) / eta
            R = R - np.outer(y, Rl) / eta
            R[l] = 0.0
            occ[l] = False
            slot_row[l] = -1
            u[l] = 0.0
            drops += 1
            cost += 0.6   # H R_l, R (H R_l): two matvecs, two more barriers
    return dict(passes=passes, it=it, drops=drops, multi=multi, x=x, cost=cost, active=sorted(slot_row[occ].tolist()),
                u=u[occ])


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    ks = [a for a in sys.argv[2:]] or ["1", "2", "3", "4"]
    N = int(os.environ.get("GI_N", "10"))   # GI_N=16 GI_GAITS=trot10,pace10,bound8: the config-4 mix
    bt = make_batch(B, N, seed=1000, gaits=tuple(os.environ.get("GI_GAITS", "trot10").split(",")), robots=("a1",))
    qps = [robot_qp(bt, b, N) for b in range(B)]
    ref = None
    for ka in ks:
        parts = ka.split(":")   # "k", "k:ratio" or "k:ratio:drops"
        k, r = int(parts[0]), float(parts[1]) if len(parts) > 1 else 0.0
        sd = int(parts[2]) if len(parts) > 2 else 10**9
        res = [simulate(*qp, kmax=k, ratio=r, stop_after_drops=sd, metric=os.environ.get("GI_METRIC", "P"))
               for qp in qps]
        passes = np.array([r["passes"] for r in res])
        its = np.array([r["it"] for r in res])
        drops = np.array([r["drops"] for r in res])
        if ref is None:
            ref = [r["x"] for r in res]
        cost = np.array([r["cost"] for r in res])
        dev = max(np.abs(r["x"] - x0).max() / max(np.abs(x0).max(), 1e-3) for r, x0 in zip(res, ref))
        top = np.argsort(passes)[-5:]
        print(f"k={ka}: passes mean {passes.mean():.1f} max {passes.max()} | it mean {its.mean():.1f} max {its.max()}"
              f" | drops mean {drops.mean():.2f} max {drops.max()} | x dev vs k={ks[0]} {dev:.1e}"
              f" | cost mean {cost.mean():.1f} max {cost.max():.1f}"
              f" | slowest {[(int(i), int(passes[i]), int(its[i]), int(drops[i])) for i in top]}")


if __name__ == "__main__":
    main()
