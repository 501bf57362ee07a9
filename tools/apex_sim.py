"""Diagnostic (CPU): the engine's dual active set with pair steps (tools/gi_sim.py rules)
plus an "apex block" step -- when the chosen row's foot-step force lies in the polar cone
of its pyramid (its projection onto the cone is the apex f = 0, with a cosine margin
DELTA to the pyramid's edges), try adding three of the foot's face rows at once (each
3-subset, accepted when every multiplier stays positive, as a pair step is).
Usage: python tools/apex_sim.py [B] [DELTA]      Results: DESIGN.md section 9."""
import itertools
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), ROOT, os.path.join(ROOT, "pympc-quadruped_amd")]
from gi_sim import robot_qp
from scipy.optimize import nnls
from mpcqp.synthetic import make_batch

DELTA = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
def simulate(H, g, A, b, foot, apex=True, tol=1e-9, max_pass=2000):
    n = H.shape[0]
    W = np.linalg.inv(H); P = W.copy(); R = np.zeros((n, n))
    occ = np.zeros(n, bool); slot_row = -np.ones(n, int); u = np.zeros(n)
    x = -W @ g
    wscale = np.max(np.diag(W))
    passes = it = drops = apexes = 0
    p = -1; up = 0.0
    def try_block(cands, s):
        nonlocal x, u, P, R, occ, slot_row, it
        Z = P @ A[cands].T; Rk = R @ A[cands].T; Sk = A[cands] @ Z
        k = len(cands)
        if np.linalg.matrix_rank(Sk) < k or np.min(np.linalg.eigvalsh(0.5*(Sk+Sk.T))) <= 1e-12 * wscale:
            return False
        t = -np.linalg.solve(Sk, s[cands])
        if np.any(t <= 0): return False
        unew = u - Rk @ t
        if np.any(unew[occ] < 0): return False
        x = x + Z @ t; u = np.where(occ, unew, u)
        free = np.flatnonzero(~occ)[:k]
        E = np.zeros((n, k)); E[free, np.arange(k)] = 1.0
        Si = np.linalg.inv(Sk)
        P = P - Z @ Si @ Z.T; R = R - (Rk - E) @ Si @ Z.T
        for j, q in enumerate(free):
            occ[q] = True; slot_row[q] = cands[j]; u[q] = t[j]
        it += k
        return True
    while passes < max_pass:
        s = A @ x - b
        s[slot_row[occ]] = np.inf
        if p < 0:
            scale = 1.0 / np.sqrt(np.maximum(np.einsum("ij,jk,ik->i", A, P, A), 1e-9 * wscale))
            key = np.where(s < -tol, s * scale, np.inf)
            if not np.isfinite(key.min()): break
            order = np.argsort(key, kind="stable")
            p = order[0]; up = 0.0
            passes += 1
            j = foot[p]
            rows_j = np.flatnonzero(foot == j)
            if apex and not np.any(occ[np.isin(slot_row, rows_j)] if occ.any() else False):
                fj = x[3*j:3*j+3]
                faces = A[rows_j][:4, 3*j:3*j+3]   # the 4 pyramid faces: +-t + mu n
                nv = -A[rows_j][4, 3*j:3*j+3]      # row 4 is -n (fz <= ub)
                tt1 = 0.5 * (faces[0] - faces[1]); tt2 = 0.5 * (faces[2] - faces[3])
                mu = float(np.dot(0.5 * (faces[0] + faces[1]), nv))
                gens = [nv + mu * (s1 * tt1 + s2 * tt2) for s1 in (1, -1) for s2 in (1, -1)]
                cosmax = max(float(fj @ gk) / (np.linalg.norm(gk) * max(np.linalg.norm(fj), 1e-300)) for gk in gens)
                if cosmax < -DELTA:
                    done = False
                    for sub in itertools.combinations(range(4), 3):
                        cands = [rows_j[r] for r in sub]
                        if try_block(cands, s):
                            apexes += 1; p = -1; done = True; break
                    if done: continue
            # pair partner: best of another foot
            p2 = next((c for c in order[1:] if np.isfinite(key[c]) and foot[c] != foot[p]), None)
            if p2 is not None and try_block([p, p2], s):
                p = -1; continue
        else:
            passes += 1
        it += 1
        z = P @ A[p]; r = R @ A[p]; zsp = A[p] @ z; sp = A[p] @ x - b[p]
        thr = 1e-12 * (A[p] ** 2).sum() * wscale
        ratios = np.where(occ & (r > 0), u / np.where(r > 0, r, 1), np.inf)
        l = int(np.argmin(ratios)); t1 = ratios[l]
        t2 = -sp / zsp if zsp > thr else np.inf
        tstep = min(t1, t2)
        if np.isfinite(t2): x = x + tstep * z
        u = np.where(occ, u - tstep * r, u); up += tstep
        if t2 <= t1:
            q = int(np.flatnonzero(~occ)[0]); e = np.zeros(n); e[q] = 1.0
            P = P - np.outer(z, z) / zsp; R = R - np.outer(r - e, z) / zsp
            occ[q] = True; slot_row[q] = p; u[q] = up; p = -1
        else:
            Rl = R[l].copy(); y = R @ (H @ Rl); eta = y[l]
            P = P + np.outer(Rl, Rl) / eta; R = R - np.outer(y, Rl) / eta
            R[l] = 0.0; occ[l] = False; slot_row[l] = -1; u[l] = 0.0; drops += 1
    return dict(passes=passes, it=it, drops=drops, apexes=apexes, x=x)

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
bt = make_batch(B, 10, seed=1000, gaits=("trot10",), robots=("a1",))
res0, res1 = [], []
dev = 0
for b in range(B):
    qp = robot_qp(bt, b, 10)
    r0 = simulate(*qp, apex=False); r1 = simulate(*qp, apex=True)
    res0.append((r0["passes"], r0["it"], r0["drops"])); res1.append((r1["passes"], r1["it"], r1["drops"], r1["apexes"]))
    dev = max(dev, np.abs(r0["x"] - r1["x"]).max() / max(np.abs(r0["x"]).max(), 1e-3))
a0, a1 = np.array(res0), np.array(res1)
print("pairs     : passes mean %.1f max %d | drops mean %.2f max %d" % (a0[:,0].mean(), a0[:,0].max(), a0[:,2].mean(), a0[:,2].max()))
print("pairs+apex: passes mean %.1f max %d | drops mean %.2f max %d | apex blocks mean %.2f | x dev %.1e" % (a1[:,0].mean(), a1[:,0].max(), a1[:,2].mean(), a1[:,2].max(), a1[:,3].mean(), dev))
top = np.argsort(a0[:,0])[-6:]
print("slowest (pairs -> pairs+apex):", [(int(i), int(a0[i,0]), int(a1[i,0])) for i in top])
top1 = np.argsort(a1[:,0])[-8:]
print("slowest with apex:", [(int(i), int(a0[i,0]), int(a1[i,0]), int(a1[i,2]), int(a1[i,3])) for i in top1])
print("hist of pass change:", np.histogram(a1[:,0]-a0[:,0], bins=[-40,-10,-5,-1,0,1,5,10,40])[0])
