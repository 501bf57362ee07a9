"""Diagnostic: where the class-64 workgroups' two waves land (XCC, SE, SH, CU, SIMD),
from the stamps build's per-wave HW_ID slots.  Usage: python tools/simd_map.py [B]"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.argv = sys.argv[:2] + ["10", "trot10"]
import phase_stamps  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    slots = phase_stamps.run_raw(B, 10, ("trot10",), 1000)
    hw = slots[:, 16:18]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = (hw >> 32) & 15
    bid = (hw >> 40) & 0xffffff
    print("pairs (simd w0, simd w1):", collections.Counter(zip(simd[:, 0].tolist(), simd[:, 1].tolist())))
    key = list(zip(xcc[:, 0].tolist(), se[:, 0].tolist(), sh[:, 0].tolist(), cu[:, 0].tolist()))
    groups = collections.defaultdict(list)
    for b in range(B):
        groups[key[b]].append((int(bid[b, 0]), int(simd[b, 0]), int(simd[b, 1])))
    print("CUs:", len(groups), "robots per CU:", collections.Counter(len(v) for v in groups.values()))
    pat = collections.Counter()
    for k, v in list(groups.items()):
        v.sort()
        pat[tuple((w0, w1) for _, w0, w1 in v)] += 1
    for p, c in pat.most_common(12):
        print(c, p)
    for k, v in list(groups.items())[:6]:
        print(k, v)
    print("xcc vs bid%8:", collections.Counter(zip(xcc[:, 0].tolist(), (bid[:, 0] % 8).tolist())).most_common(10))


if __name__ == "__main__":
    main()
