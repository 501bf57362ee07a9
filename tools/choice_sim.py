"""Diagnostic (CPU): the kernel's pair-step dual active set (tools/gi_sim.py rules) with
row-choice variants that favour foot-steps already holding active rows -- "foot:b" scales
the key of rows of such foot-steps by 1 + b, "foot2:b" only when they hold two, "pair:b"
only for the pair partner.  Per-batch maximum passes on the benchmark's config-2 batches:
    python tools/choice_sim.py 1024 <seed> foot:0,foot:0.3,pair:0.5
Results: DESIGN.md section 4.5 (round 4)."""
import sys, os, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), ROOT, os.path.join(ROOT, "pympc-quadruped_amd")]
from gi_sim import robot_qp
from mpcqp.synthetic import make_batch

def simulate(H, g, A, b, foot, bonus=0.0, tol=1e-9, max_pass=2000, mode="foot"):
    n = H.shape[0]
    W = np.linalg.inv(H); P = W.copy(); R = np.zeros((n, n))
    occ = np.zeros(n, bool); slot_row = -np.ones(n, int); u = np.zeros(n)
    x = -W @ g
    wscale = np.max(np.diag(W))
    passes = it = drops = 0
    p = -1; up = 0.0
    nf = foot.max() + 1
    while passes < max_pass:
        s = A @ x - b
        s[slot_row[occ]] = np.inf
        if p < 0:
            scale = 1.0 / np.sqrt(np.maximum(np.einsum("ij,jk,ik->i", A, P, A), 1e-9 * wscale))
            key = np.where(s < -tol, s * scale, np.inf)
            if not np.isfinite(key.min()): break
            if bonus:
                cnt = np.zeros(nf, int)
                for r in slot_row[occ]: cnt[foot[r]] += 1
                if mode == "foot":
                    key = np.where(np.isfinite(key) & (cnt[foot] > 0), key * (1 + bonus), key)
                elif mode == "foot2":
                    key = np.where(np.isfinite(key) & (cnt[foot] > 1), key * (1 + bonus), key)
                elif mode == "pair":
                    key2 = np.where(np.isfinite(key) & (cnt[foot] > 0), key * (1 + bonus), key)
                elif mode == "fresh":
                    key = np.where(np.isfinite(key) & (cnt[foot] == 0), key * (1 + bonus), key)
            order = np.argsort(key, kind="stable")
            p = order[0]; up = 0.0
            passes += 1
            if bonus and mode == "pair":
                o2 = np.argsort(key2, kind="stable")
                p2 = next((c for c in o2 if np.isfinite(key2[c]) and foot[c] != foot[p]), None)
            else:
                p2 = next((c for c in order[1:] if np.isfinite(key[c]) and foot[c] != foot[p]), None)
            if p2 is not None:
                cands = [p, p2]
                Z = P @ A[cands].T; Rk = R @ A[cands].T; Sk = A[cands] @ Z
                ok = np.min(np.linalg.eigvalsh(0.5 * (Sk + Sk.T))) > 1e-12 * wscale
                if ok:
                    t = -np.linalg.solve(Sk, s[cands])
                    unew = u - Rk @ t
                    if np.all(t > 0) and not np.any(unew[occ] < 0):
                        x = x + Z @ t; u = np.where(occ, unew, u)
                        free = np.flatnonzero(~occ)[:2]
                        E = np.zeros((n, 2)); E[free, np.arange(2)] = 1.0
                        Si = np.linalg.inv(Sk)
                        P = P - Z @ Si @ Z.T; R = R - (Rk - E) @ Si @ Z.T
                        for j, q in enumerate(free):
                            occ[q] = True; slot_row[q] = cands[j]; u[q] = t[j]
                        it += 2; p = -1
                        continue
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
    return passes, it, drops, x

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
bt = make_batch(B, 10, seed=seed, gaits=("trot10",), robots=("a1",))
qps = [robot_qp(bt, b, 10) for b in range(B)]
ref = None
VARS = [(v.split(":")[0], float(v.split(":")[1])) for v in sys.argv[3].split(",")]
for mode, bonus in VARS:
    res = [simulate(*qp, bonus=bonus, mode=mode) for qp in qps]
    pa = np.array([r[0] for r in res]); it = np.array([r[1] for r in res]); dr = np.array([r[2] for r in res])
    if ref is None: ref = [r[3] for r in res]
    dev = max(np.abs(r[3] - x0).max() / max(np.abs(x0).max(), 1e-3) for r, x0 in zip(res, ref))
    top = np.argsort(pa)[-4:]
    print(f"{mode} bonus {bonus}: passes mean {pa.mean():.1f} max {pa.max()} p99 {np.percentile(pa,99):.0f} | it mean {it.mean():.1f} max {it.max()} | drops max {dr.max()} | dev {dev:.1e} | top {[(int(i), int(pa[i])) for i in top]}", flush=True)
