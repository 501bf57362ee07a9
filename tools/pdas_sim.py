"""Diagnostic: alternatives to the engine's dual active set, simulated on the CPU over a
seeded config-2 batch (python tools/pdas_sim.py [B]).

* Warm starts of the projected GI loop (`gi_sim.simulate(init_rows=...)`): the rows
  violated at the unconstrained optimum, or each foot-step's own cone projection (in its
  3x3 block of W), reduced until every multiplier is >= 0.
* The primal-dual active-set method (PDAS: next set = {active rows with lambda > 0} U
  {violated rows}; each iteration an equality-constrained solve), counted in iterations,
  row additions / removals and rank-deficient sets, and priced with a pass cost model:
  cycles per incremental add / drop / iteration against a GI pass, taken from the
  B = 1024 section stamps (profiles/r2_v5/r2_v5_stamps_c2.txt).
Results: DESIGN.md §4.5.
"""
import itertools
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), ROOT, os.path.join(ROOT, "pympc-quadruped_amd")]
from gi_sim import robot_qp, simulate  # noqa: E402
from mpcqp.synthetic import make_batch  # noqa: E402

ADD, DROP, ITER, GIPASS = 2000, 3500, 3000, 6600   # cycles (cost model, see docstring)


def dual_feasible(H, g, A, b, G):
    """Drop the most negative multiplier until the equality-constrained optimum on G has lambda >= 0."""
    W = np.linalg.inv(H)
    xu = -W @ g
    G = list(G)
    while G:
        AG = A[G]
        lam = np.linalg.lstsq(AG @ W @ AG.T, b[G] - AG @ xu, rcond=None)[0]
        if np.all(lam >= 0):
            break
        G.pop(int(np.argmin(lam)))
    return G


def guess_violated(H, g, A, b, foot):
    x = -np.linalg.solve(H, g)
    return list(np.flatnonzero(A @ x - b < -1e-9))


def guess_per_foot(H, g, A, b, foot):
    """Each violated foot-step's force projected onto its own cone (metric: its block of W)."""
    W = np.linalg.inv(H)
    x = -W @ g
    G = []
    for j in range(len(x) // 3):
        rows = np.flatnonzero(foot == j)
        a, bb, f0 = A[rows][:, 3 * j:3 * j + 3], b[rows], x[3 * j:3 * j + 3]
        if np.all(a @ f0 - bb >= -1e-9):
            continue
        Wj = W[3 * j:3 * j + 3, 3 * j:3 * j + 3]
        found = None
        for k in (1, 2, 3):
            for sub in itertools.combinations(range(len(rows)), k):
                aS = a[list(sub)]
                Ms = aS @ Wj @ aS.T
                if abs(np.linalg.det(Ms)) < 1e-14:
                    continue
                lam = np.linalg.solve(Ms, bb[list(sub)] - aS @ f0)
                if np.all(lam >= -1e-12) and np.all(a @ (f0 + Wj @ aS.T @ lam) - bb >= -1e-9):
                    found = sub
                    break
            if found is not None:
                break
        if found is not None:
            G += [int(rows[i]) for i in found]
    return G


def pdas(H, g, A, b, foot, maxit=60):
    W = np.linalg.inv(H)
    xu = -W @ g
    m = len(b)
    act = np.zeros(m, bool)
    x, lam = xu, np.zeros(m)
    adds = drops = dep = 0
    for it in range(1, maxit + 1):
        s = A @ x - b
        new = np.where(act, lam > 1e-12, s < -1e-9)
        if np.array_equal(new, act):
            ok = bool(np.all(s >= -1e-7) and np.all(lam >= -1e-9))
            return dict(it=it, adds=adds, drops=drops, ok=ok, x=x, dep=dep)
        adds += int((new & ~act).sum())
        drops += int((act & ~new).sum())
        act = new
        G = np.flatnonzero(act)
        AG = A[G]
        M = AG @ W @ AG.T
        if np.linalg.matrix_rank(M) < len(G):   # e.g. all pyramid faces of a foot at its apex
            dep += 1
        lg = np.linalg.lstsq(M, b[G] - AG @ xu, rcond=None)[0]
        x = xu + W @ AG.T @ lg
        lam = np.zeros(m)
        lam[G] = lg
    return dict(it=maxit, adds=adds, drops=drops, ok=False, x=x, dep=dep)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    N = 10
    bt = make_batch(B, N, seed=1000, gaits=("trot10",), robots=("a1",))
    qps = [robot_qp(bt, b, N) for b in range(B)]
    cold = [simulate(*qp, kmax=2) for qp in qps]
    p0 = np.array([r["passes"] for r in cold])
    na = np.array([len(r["active"]) for r in cold])
    print(f"B={B} cold GI (pair steps): passes mean {p0.mean():.1f} max {p0.max()}; "
          f"final active rows mean {na.mean():.1f} max {na.max()}")
    for name, guess in (("violated at x_unc", guess_violated), ("per-foot projection", guess_per_foot)):
        res = []
        for qp, r0 in zip(qps, cold):
            G = dual_feasible(*qp[:4], guess(*qp))
            res.append((simulate(*qp, kmax=2, init_rows=G)["passes"], len(G), len(set(G) & set(r0["active"]))))
        a = np.array(res)
        print(f"warm GI ({name}): passes mean {a[:, 0].mean():.1f} max {a[:, 0].max()} | "
              f"guess size mean {a[:, 1].mean():.1f}, of them in the final set {a[:, 2].mean():.1f}")
    rows = []
    for qp, r0 in zip(qps, cold):
        r = pdas(*qp)
        dev = np.abs(r["x"] - r0["x"]).max() / max(np.abs(r0["x"]).max(), 1e-3)
        rows.append((r["it"], r["adds"], r["drops"], r["ok"], r["dep"], dev,
                     r["adds"] * ADD + r["drops"] * DROP + r["it"] * ITER, r0["passes"] * GIPASS))
    a = np.array(rows, dtype=float)
    print(f"PDAS: iterations mean {a[:, 0].mean():.1f} max {int(a[:, 0].max())} | adds mean {a[:, 1].mean():.1f} "
          f"max {int(a[:, 1].max())} | removals mean {a[:, 2].mean():.1f} max {int(a[:, 2].max())} | "
          f"converged {int(a[:, 3].sum())}/{B} | rank-deficient sets {int(a[:, 4].sum())} | x dev {a[:, 5].max():.1e}")
    print(f"cost model (cycles): GI mean {a[:, 7].mean():.0f} max {a[:, 7].max():.0f} | "
          f"PDAS mean {a[:, 6].mean():.0f} max {a[:, 6].max():.0f}")


if __name__ == "__main__":
    main()
