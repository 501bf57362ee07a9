"""Diagnostic (round 5): the dispatch-order key of mpcqp_order_kernel (csrc/mpcqp.hip).

A robot's solve time follows its active-set iteration count.  This script measures, on the
bench's seeded batches, how well the key |v0 - vref_0| (horizontal velocity error, the
correction the cone forces must supply) predicts that count, and what ordering the batch by it
does to a queueing launch: each CU takes the next robot (in workgroup order) when its current
one ends, with the robot's cost = setup + per-iteration cost x its iteration count (the
kernel's own iteration counts replayed by tools/gi_sim.py).
Usage: python tools/order_sim.py [B] [N] [gaits] [slots]
  config 2: 1024 10 trot10 1024    config 4: 2048 16 trot10,pace10,bound8 256
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gi_sim import robot_qp, simulate  # noqa: E402
from mpcqp.synthetic import make_batch  # noqa: E402


def makespan(cost, order, slots):
    """Greedy list schedule: robots in `order` go to the first free slot."""
    free = np.zeros(slots)
    for r in order:
        k = int(np.argmin(free))
        free[k] += cost[r]
    return free.max()


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    gaits = tuple(sys.argv[3].split(",")) if len(sys.argv) > 3 else ("trot10",)
    slots = int(sys.argv[4]) if len(sys.argv) > 4 else 256
    bt = make_batch(B, N, seed=1000, gaits=gaits, robots=("a1",))
    it = np.array([simulate(*robot_qp(bt, b, N), kmax=2)["it"] for b in range(B)], float)
    x0, xr = bt["x0"], bt["xref"].reshape(B, N, 13)
    key = np.hypot(x0[:, 9] - xr[:, 0, 9], x0[:, 10] - xr[:, 0, 10])
    print(f"B={B} N={N} {'+'.join(gaits)}: iterations mean {it.mean():.1f} max {it.max():.0f}; "
          f"corr(key, iterations) {np.corrcoef(key, it)[0, 1]:.3f}")
    top = np.argsort(it)[-20:]
    rank = np.argsort(np.argsort(-key))
    print("  key ranks of the 20 slowest robots:", sorted(rank[top].tolist()))
    # cost model: a setup of S iterations' worth plus one unit per iteration
    for setup in (10.0, 25.0):
        cost = setup + it
        base = makespan(cost, np.arange(B), slots)
        srt = makespan(cost, np.argsort(-key, kind="stable"), slots)
        ideal = makespan(cost, np.argsort(-cost, kind="stable"), slots)
        print(f"  setup = {setup:.0f} iterations, {slots} slots: makespan batch order {base:.0f}, key order {srt:.0f} "
              f"({(1 - srt / base) * 100:+.1f} %), exact-cost order {ideal:.0f} ({(1 - ideal / base) * 100:+.1f} %), "
              f"mean load {cost.sum() / slots:.0f}")


if __name__ == "__main__":
    main()
