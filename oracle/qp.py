"""CPU oracle, part 2: exact float64 solvers for the Drake-branch QP
(TEST INFRASTRUCTURE ONLY -- imported by tests/, smoke() and bench.py's
cpu_baseline leg, never by the product path).

The reference solves (mpc.py:277-286, Drake ``MathematicalProgram``)

    min_U  1/2 U^T H U + g^T U     s.t.  lb <= C U <= ub

with Drake's ``AddQuadraticCost(Q, b)`` meaning 1/2 x^T Q x + b^T x.  Drake
1.15.0 (requirements.txt:23) picks its solver at run time and is not
installed here; its answer cannot be reproduced bit-for-bit.  The problem is
strictly convex (H >= 2 Rbar = 2e-5 I) and always feasible (U = 0), so its
optimum is unique: the oracle is that optimum, computed two independent ways
and certified by KKT residuals.

* ``solve_qp_dual_active_set`` -- Goldfarb-Idnani dual active-set method on
  the raw two-sided problem (every row of C, swing rows included), float64,
  Householder/Givens updates of J = L^{-T}.  Exact up to float64 rounding.
* ``solve_qp_interior_point`` -- Mehrotra primal-dual interior point on the
  swing-eliminated problem (swing GRFs are provably 0: ub gives fz <= 0, the
  cone rows give mu*fz >= |fx|, |fy| >= 0), used only to cross-check.
* ``kkt_residuals`` -- stationarity / primal / dual / complementarity.
"""
import numpy as np


def _one_sided(C, lb, ub):
    """lb <= C x <= ub  ->  A x >= b (finite sides only)."""
    C = np.asarray(C, dtype=np.float64)
    lb = np.asarray(lb, dtype=np.float64)
    ub = np.asarray(ub, dtype=np.float64)
    rows, rhs, src, sign = [], [], [], []
    for i in range(C.shape[0]):
        if np.isfinite(lb[i]):
            rows.append(C[i]); rhs.append(lb[i]); src.append(i); sign.append(1.0)
        if np.isfinite(ub[i]):
            rows.append(-C[i]); rhs.append(-ub[i]); src.append(i); sign.append(-1.0)
    return np.array(rows), np.array(rhs), np.array(src), np.array(sign)


def solve_qp_dual_active_set(H, g, C, lb, ub, max_iter=10000, tol=1e-11):
    """Goldfarb-Idnani (Math. Prog. 27, 1983) dual active-set, float64.

    Returns (x, y, info) where y are the two-sided multipliers per row of C
    (y > 0: lower bound active, y < 0: upper bound active) so that
    H x + g = C^T y at the optimum.
    """
    G = np.asarray(H, dtype=np.float64)
    a = np.asarray(g, dtype=np.float64)
    A, b, src, sgn = _one_sided(C, lb, ub)
    n = G.shape[0]
    L = np.linalg.cholesky(G)
    J = np.linalg.inv(L).T                      # J^T G J = I
    x = -np.linalg.solve(G, a)                  # unconstrained minimiser
    R = np.zeros((n, n))
    active = []                                 # indices into A
    u = np.zeros(0)
    it = 0
    scale = 1.0 + np.abs(b).max(initial=0.0)
    rounding_accept = []   # (row, its multiplier, the largest violation) of a rounding-level stop
    while True:
        s = A @ x - b
        p = int(np.argmin(s)) if len(s) else -1
        if p < 0 or s[p] >= -tol * scale:
            break
        npv = A[p]
        u_p = 0.0
        done = False
        while True:
            it += 1
            if it > max_iter:
                raise RuntimeError("dual active set: iteration limit")
            q = len(active)
            d = J.T @ npv
            z = J[:, q:] @ d[q:]
            r = np.linalg.solve(np.triu(R[:q, :q]), d[:q]) if q else np.zeros(0)
            # dual (partial) step: largest t keeping active multipliers >= 0
            t1, l_drop = np.inf, -1
            for j in range(q):
                if r[j] > 0:
                    ratio = u[j] / r[j]
                    if ratio < t1:
                        t1, l_drop = ratio, j
            # primal (full) step
            zn = float(z @ npv)
            dn = float(d @ d)
            if zn > 1e-14 * max(dn, 1e-300):
                t2 = -(float(npv @ x) - b[p]) / zn
            else:
                t2 = np.inf
            t = min(t1, t2)
            if not np.isfinite(t):
                # p is dependent on the active set and no multiplier can move.  In exact
                # arithmetic that is infeasibility, which the MPC QP cannot have (U = 0 is
                # feasible); a violation at rounding level (a flight schedule's forced-zero
                # GRFs at N = 32: s = -3e-11 against dn = 4e4) is rounding noise of the
                # J / R updates.  Accepted only when EVERY row, re-evaluated at the current x
                # (earlier partial steps for p have moved it), is satisfied to 1e-8 * scale;
                # p then keeps the multiplier u_p its partial steps gave it (stationarity
                # H x + g = A^T u + u_p a_p holds throughout), reported in y and in info.
                s_now = A @ x - b
                if (-s_now).max(initial=0.0) <= 1e-8 * scale:
                    rounding_accept.append((p, u_p, float(-s_now.min(initial=0.0))))
                    done = True
                    break
                raise RuntimeError("QP infeasible (cannot happen for the MPC QP)")
            if not np.isfinite(t2):
                # pure dual step: constraint p is dependent on the active set
                u = u - t * r
                u_p += t
                R, J, active, u = _drop(R, J, active, u, l_drop)
                continue
            x = x + t * z
            u = u - t * r
            u_p += t
            if t == t2:
                # add p: rotate d[q:] onto e_q (Householder), extend R
                R, J = _add(R, J, d, q)
                active.append(p)
                u = np.append(u, u_p)
                break
            R, J, active, u = _drop(R, J, active, u, l_drop)
        if done:
            break
    y = np.zeros(np.asarray(C).shape[0])
    for k, j in enumerate(active):
        y[src[j]] += sgn[j] * u[k]
    for j, up, _ in rounding_accept:
        y[src[j]] += sgn[j] * up
    return x, y, dict(iterations=it, active=[(int(src[j]), int(sgn[j])) for j in active],
                      rounding_accept=[(int(src[j]), float(up), v) for j, up, v in rounding_accept])


def _add(R, J, d, q):
    n = J.shape[0]
    v = d[q:].copy()
    alpha = np.linalg.norm(v)
    if q < n - 1 and alpha > 0:
        sign = 1.0 if v[0] >= 0 else -1.0
        v[0] += sign * alpha
        vv = float(v @ v)
        if vv > 0:
            J[:, q:] -= np.outer(J[:, q:] @ v, v) * (2.0 / vv)
        r_qq = -sign * alpha
    else:
        r_qq = v[0] if len(v) else 0.0
    R = R.copy()
    R[:q, q] = d[:q]
    R[q, q] = r_qq
    return R, J


def _drop(R, J, active, u, l):
    q = len(active)
    R = np.delete(R[:q, :q], l, axis=1)         # q x (q-1), Hessenberg from column l
    for j in range(l, q - 1):
        a_, b_ = R[j, j], R[j + 1, j]
        h = np.hypot(a_, b_)
        if h == 0:
            continue
        c, s = a_ / h, b_ / h
        Rj, Rj1 = R[j, :].copy(), R[j + 1, :].copy()
        R[j, :] = c * Rj + s * Rj1
        R[j + 1, :] = -s * Rj + c * Rj1
        Jj, Jj1 = J[:, j].copy(), J[:, j + 1].copy()
        J[:, j] = c * Jj + s * Jj1
        J[:, j + 1] = -s * Jj + c * Jj1
    n = J.shape[0]
    Rn = np.zeros((n, n))
    Rn[:q - 1, :q - 1] = np.triu(R[:q - 1, :q - 1])
    active = active[:l] + active[l + 1:]
    u = np.delete(u, l)
    return Rn, J, active, u


def swing_elimination(contact, horizon):
    """Indices of the free (stance) variables of U; the rest are exactly 0."""
    contact = np.asarray(contact).reshape(-1)
    idx = []
    for k in range(4 * horizon):
        if contact[k] > 0:
            idx.extend([3 * k, 3 * k + 1, 3 * k + 2])
    return np.array(idx, dtype=np.int64)


def solve_qp_interior_point(H, g, C, lb, ub, contact, horizon, tol=1e-13, max_iter=200):
    """Mehrotra predictor-corrector IPM on the swing-eliminated problem (cross-check)."""
    idx = swing_elimination(contact, horizon)
    n_full = H.shape[0]
    x_full = np.zeros(n_full)
    if len(idx) == 0:
        return x_full
    Hr = np.asarray(H, dtype=np.float64)[np.ix_(idx, idx)]
    gr = np.asarray(g, dtype=np.float64)[idx]
    # rows of C touching only stance variables (swing rows are identically 0 <= 0 <= ub)
    rows = [r for r in range(C.shape[0]) if np.any(C[r, idx] != 0)]
    Cr = np.asarray(C, dtype=np.float64)[np.ix_(rows, idx)]
    A, b, _, _ = _one_sided(Cr, np.asarray(lb)[rows], np.asarray(ub)[rows])
    m, n = A.shape
    x = np.zeros(n)
    # strictly interior start: small positive fz
    for k in range(0, n, 3):
        x[k + 2] = 1.0
    s = np.maximum(A @ x - b, 1.0)
    lam = np.ones(m)
    for _ in range(max_iter):
        rd = Hr @ x + gr - A.T @ lam
        rp = A @ x - b - s
        mu = s @ lam / m
        if (np.linalg.norm(rd, np.inf) < tol * (1 + np.abs(gr).max())
                and np.linalg.norm(rp, np.inf) < tol * (1 + np.abs(b).max()) and mu < tol):
            break

        def newton(rc):
            # H dx - A^T dl = -rd ; A dx - ds = -rp ; Lam ds + S dl = rc
            # => (H + A^T W A) dx = -rd + A^T (S^-1 rc - W rp),  W = Lam / S
            w = lam / s
            K = Hr + A.T @ (w[:, None] * A)
            rhs = -rd + A.T @ (w * (-rp) + rc / s)
            dx = np.linalg.solve(K, rhs)
            ds = A @ dx + rp
            dl = (rc - lam * ds) / s
            return dx, ds, dl

        # predictor (affine)
        dx, ds, dl = newton(-s * lam)
        a_p = _max_step(s, ds)
        a_d = _max_step(lam, dl)
        mu_aff = (s + a_p * ds) @ (lam + a_d * dl) / m
        sigma = (mu_aff / mu) ** 3
        dx, ds, dl = newton(-s * lam - ds * dl + sigma * mu)
        a_p = min(1.0, 0.995 * _max_step(s, ds))
        a_d = min(1.0, 0.995 * _max_step(lam, dl))
        x += a_p * dx
        s += a_p * ds
        lam += a_d * dl
    x_full[idx] = x
    return x_full


def _max_step(v, dv):
    neg = dv < 0
    if not np.any(neg):
        return 1.0
    return float(min(1.0, np.min(-v[neg] / dv[neg])))


def kkt_residuals(H, g, C, lb, ub, x, y):
    """Scaled KKT residuals of (x, y) for lb <= Cx <= ub (y: two-sided multipliers)."""
    H = np.asarray(H, dtype=np.float64)
    C = np.asarray(C, dtype=np.float64)
    lb = np.asarray(lb, dtype=np.float64)
    ub = np.asarray(ub, dtype=np.float64)
    cx = C @ x
    stat = np.abs(H @ x + g - C.T @ y).max()
    prim = max(np.maximum(lb - cx, 0).max(), np.maximum(cx - ub, 0).max())
    dual = max(np.maximum(-y[np.isinf(ub)], 0).max(initial=0.0), 0.0)
    ubf = np.where(np.isfinite(ub), ub, 0.0)
    comp = max(np.abs(np.maximum(y, 0) * (cx - lb)).max(),
               np.abs(np.minimum(y, 0) * np.where(np.isfinite(ub), ubf - cx, 0.0)).max())
    return dict(stationarity=float(stat), primal=float(prim), dual=float(dual),
                complementarity=float(comp))
