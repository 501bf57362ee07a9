"""Diagnostic (round 5): what four robots per CU cost each robot of a config-2 batch.

Runs the same seeded batch through two stamps builds (-DMPCQP_STAMPS): the shipped launch (four
class-64 robots per CU) and one with 96 KB of extra dynamic LDS per workgroup
(-DMPCQP_SOLO_LDS=98304: one robot per CU, the batch in four rounds), and compares every
robot's own cycle count (s_memtime from its first to its last stamp).  The slowest robots'
ratio is the most the co-residency lever could give the launch.
  build:  python tools/solo_stamps.py build
  run:    python tools/solo_stamps.py [B]
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOLO = os.path.join(ROOT, "tools", "libmpcqp_stamps_solo.so")
SHARED = os.path.join(ROOT, "pympc-quadruped_amd", "mpcqp", "libmpcqp_stamps.so")

if len(sys.argv) > 1 and sys.argv[1] == "build":
    src = os.path.join(ROOT, "pympc-quadruped_amd", "csrc", "mpcqp.hip")
    base = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
            "-DMPCQP_STAMPS", "-I" + os.path.join(ROOT, "include")]
    subprocess.run(base + ["-o", SHARED, src], check=True)
    subprocess.run(base + ["-DMPCQP_SOLO_LDS=98304", "-o", SOLO, src], check=True)
    sys.exit(0)

sys.path.insert(0, os.path.join(ROOT, "tools"))


def one(lib, B, out):
    """One stamps build in this process (the library is loaded once per process)."""
    os.environ["MPCQP_STAMPS_LIB"] = lib
    import phase_stamps
    slots, it = phase_stamps.run_raw(B, 10, ("trot10",), 1000, with_iters=True)
    ts = slots[:, :7]
    np.savez(out, cyc=ts[:, 6] - ts[:, 0], it=it)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "one":
        one(sys.argv[2], int(sys.argv[3]), sys.argv[4])
        return
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    res = []
    for lib, tag in ((SHARED, "shared"), (SOLO, "solo")):
        out = os.path.join(ROOT, "gpurun_out", f"solo_{tag}.npz")
        subprocess.run([sys.executable, __file__, "one", lib, str(B), out], check=True)
        res.append(np.load(out))
    sh, so, it = res[0]["cyc"], res[1]["cyc"], res[0]["it"]
    assert np.array_equal(it, res[1]["it"])
    r = sh / so
    print(f"B={B}: robot cycles shared/solo median {np.median(r):.2f} p90 {np.percentile(r, 90):.2f} max {r.max():.2f}")
    for i in np.argsort(sh)[-8:]:
        print(f"  robot {i}: iterations {it[i]} cycles shared {sh[i]} solo {so[i]} ratio {r[i]:.2f}")
    print(f"  slowest robot: shared {sh.max()} cycles ({sh.max() / 2.4e3:.1f} us at 2.4 GHz), the slowest solo "
          f"{so.max()} ({so.max() / 2.4e3:.1f} us): the bound a launch of these robots cannot beat")


if __name__ == "__main__":
    main()
