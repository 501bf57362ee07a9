"""Diagnostic (round 5, verdict r4 item 1): can a float32 run of the kernel's projected
Goldfarb-Idnani loop identify the active set, so that one float64 equality-constrained
solve on that set (verified by primal feasibility and multiplier signs) replaces the
float64 loop?

For every robot of the bench's seeded batches:
  1. the float64 loop (tools/gi_sim.py, the kernel's rules: current-metric keys, pair
     steps) -> x*, its active set and pass count;
  2. the same loop with every array in float32 (H^-1 by an f32 solve, P, R, x, s, u in
     f32) -> the identified set A32 (or a failure: infeasible / pass cap);
  3. the f64 polish on A32: x = argmin on {a_c . x = b_c, c in A32}, multipliers from the
     f64 KKT system; verified when every row is feasible (>= -1e-9 scale) and every
     multiplier >= 0.  A failed check is corrected (the most negative multiplier out, or
     the most violated row in) and re-solved, up to 8 times.
Gate (verdict r4): >= 99.9 % of robots verified with <= 1 correction and u0 within 1e-5
of the f64 loop's.
Usage: python tools/mp_sim.py [B] [seeds...]   (GI_N / GI_GAITS as gi_sim.py)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gi_sim import robot_qp, simulate  # noqa: E402
from mpcqp.synthetic import make_batch  # noqa: E402


def simulate_f32(H, g, A, b, foot, tol=1e-9, max_pass=600):
    """The kernel's loop (current-metric keys, pair steps) with float32 arithmetic."""
    f = np.float32
    H32, g32, A32, b32 = H.astype(f), g.astype(f), A.astype(f), b.astype(f)
    n = H.shape[0]
    try:
        W = np.linalg.solve(H32, np.eye(n, dtype=f)).astype(f)
    except np.linalg.LinAlgError:
        return None
    W = ((W + W.T) * f(0.5)).astype(f)
    P = W.copy()
    R = np.zeros((n, n), f)
    occ = np.zeros(n, bool)
    slot_row = -np.ones(n, int)
    u = np.zeros(n, f)
    x = (-W @ g32).astype(f)
    wscale = f(np.max(np.diag(W)))
    passes = 0
    p = -1
    up = f(0)
    while passes < max_pass:
        s = (A32 @ x - b32).astype(f)
        s[slot_row[occ]] = np.inf
        if p < 0:
            q = np.einsum("ij,jk,ik->i", A32, P, A32).astype(f)
            key = np.where(s < -tol, s / np.sqrt(np.maximum(q, f(1e-9) * wscale)), np.inf)
            if not np.isfinite(key.min()):
                return dict(passes=passes, active=sorted(slot_row[occ].tolist()), status="ok")
            order = np.argsort(key, kind="stable")
            p = int(order[0])
            p2 = -1
            for c in order[1:]:
                if not np.isfinite(key[c]):
                    break
                if foot[c] != foot[p]:
                    p2 = int(c)
                    break
            up = f(0)
            if p2 >= 0:   # pair step
                cands = [p, p2]
                Z = (P @ A32[cands].T).astype(f)
                Rk = (R @ A32[cands].T).astype(f)
                Sm = (A32[cands] @ Z).astype(f)
                thr = f(1e-12) * (A32[cands] ** 2).sum(1) * wscale
                det = Sm[0, 0] * Sm[1, 1] - Sm[0, 1] * Sm[1, 0]
                if Sm[0, 0] > thr[0] and Sm[1, 1] > thr[1] and det > thr[1] * Sm[0, 0]:
                    t = (-np.linalg.solve(Sm.astype(f), s[cands])).astype(f)
                    unew = (u - Rk @ t).astype(f)
                    if np.all(t > 0) and not np.any(unew[occ] < 0):
                        passes += 1
                        x = (x + Z @ t).astype(f)
                        u = np.where(occ, unew, u).astype(f)
                        free = np.flatnonzero(~occ)[:2]
                        E = np.zeros((n, 2), f)
                        E[free, np.arange(2)] = 1
                        Si = np.linalg.inv(Sm).astype(f)
                        P = (P - Z @ Si @ Z.T).astype(f)
                        R = (R - (Rk - E) @ Si @ Z.T).astype(f)
                        for j, qq in enumerate(free):
                            occ[qq] = True
                            slot_row[qq] = cands[j]
                            u[qq] = t[j]
                        p = -1
                        continue
        passes += 1
        z = (P @ A32[p]).astype(f)
        r = (R @ A32[p]).astype(f)
        zsp = f(A32[p] @ z)
        sp = f(A32[p] @ x - b32[p])
        thr = f(1e-12) * (A32[p] ** 2).sum() * wscale
        ratios = np.where(occ & (r > 0), u / np.where(r > 0, r, 1), np.inf)
        l = int(np.argmin(ratios))
        t1 = ratios[l]
        t2 = -sp / zsp if zsp > thr else np.inf
        tstep = f(min(t1, t2))
        if not np.isfinite(tstep):
            return dict(passes=passes, active=sorted(slot_row[occ].tolist()), status="infeasible")
        if np.isfinite(t2):
            x = (x + tstep * z).astype(f)
        u = np.where(occ, u - tstep * r, u).astype(f)
        up = f(up + tstep)
        if t2 <= t1:
            qq = int(np.flatnonzero(~occ)[0])
            e = np.zeros(n, f)
            e[qq] = 1
            P = (P - np.outer(z, z) / zsp).astype(f)
            R = (R - np.outer(r - e, z) / zsp).astype(f)
            occ[qq] = True
            slot_row[qq] = p
            u[qq] = up
            p = -1
        else:
            Rl = R[l].copy()
            y = (R @ (H32 @ Rl)).astype(f)
            eta = y[l]
            P = (P + np.outer(Rl, Rl) / eta).astype(f)
            R = (R - np.outer(y, Rl) / eta).astype(f)
            R[l] = 0
            occ[l] = False
            slot_row[l] = -1
            u[l] = 0
    return dict(passes=passes, active=sorted(slot_row[occ].tolist()), status="cap")


def eqp(H, g, A, b, act):
    """float64 optimum on {A_act x = b_act}: (x, multipliers)."""
    Wg = np.linalg.solve(H, g)
    x = -Wg
    if not act:
        return x, np.zeros(0)
    Aa = A[act]
    WA = np.linalg.solve(H, Aa.T)
    M = Aa @ WA
    lam = np.linalg.lstsq(M, b[act] - Aa @ x, rcond=None)[0]
    return x + WA @ lam, lam


def polish(H, g, A, b, act, max_fix=8):
    """Verify / correct an active-set guess in float64: returns (x, corrections, ok)."""
    act = list(act)
    scale = max(1.0, np.abs(b).max())
    for fix in range(max_fix + 1):
        x, lam = eqp(H, g, A, b, act)
        s = A @ x - b
        viol = s < -1e-9 * scale
        neg = lam < -1e-9 * max(1.0, np.abs(lam).max() if lam.size else 1.0)
        if not viol.any() and not neg.any():
            return x, fix, True
        if neg.any():
            act.pop(int(np.argmin(lam)))
        else:
            act.append(int(np.argmin(s)))
    return x, max_fix, False


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    seeds = [int(a) for a in sys.argv[2:]] or [1000, 2000, 3000, 4000]
    N = int(os.environ.get("GI_N", "10"))
    gaits = tuple(os.environ.get("GI_GAITS", "trot10").split(","))
    tot = 0
    fixes = []
    errs = []
    p64, p32 = [], []
    fails = {"f32 loop": 0, "unverified": 0}
    for seed in seeds:
        bt = make_batch(B, N, seed=seed, gaits=gaits, robots=("a1",))
        for rb in range(B):
            H, g, A, b, foot = robot_qp(bt, rb, N)
            ref = simulate(H, g, A, b, foot, kmax=2)
            r32 = simulate_f32(H, g, A, b, foot)
            tot += 1
            p64.append(ref["passes"])
            if r32 is None or r32["status"] != "ok":
                fails["f32 loop"] += 1
                fixes.append(99)
                continue
            p32.append(r32["passes"])
            x, nfix, ok = polish(H, g, A, b, r32["active"])
            if not ok:
                fails["unverified"] += 1
            fixes.append(nfix if ok else 99)
            # u0: the first step's stance variables (first 3 * #stance-at-step-0 entries)
            x0 = ref["x"]
            errs.append(np.abs(x[:6] - x0[:6]).max() / max(np.abs(x0[:6]).max(), 1e-3))
        print(f"seed {seed}: done", flush=True)
    fixes = np.array(fixes)
    errs = np.array(errs)
    print(f"robots {tot}: f64 passes mean {np.mean(p64):.1f} max {np.max(p64)}; f32 passes mean "
          f"{np.mean(p32):.1f} max {np.max(p32)}")
    for k in range(0, 4):
        print(f"  verified with <= {k} corrections: {(fixes <= k).mean() * 100:.2f} %")
    print(f"  f32 loop failed: {fails['f32 loop']}, unverified after 8: {fails['unverified']}")
    print(f"  u0 rel err vs the f64 loop (verified robots): max {errs.max():.2e}, "
          f"p99.9 {np.quantile(errs, 0.999):.2e}")
    gate = (fixes <= 1).mean() >= 0.999 and np.quantile(errs, 0.999) <= 1e-5
    print("GATE", "PASS" if gate else "FAIL")


if __name__ == "__main__":
    main()
