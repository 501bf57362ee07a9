"""Build libmpcqp.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "mpcqp.hip")
OUT = os.path.join(HERE, "libmpcqp.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def build(verbose=False, extra=()):
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I" + os.path.join(ROOT, "include"), "-o", OUT + ".tmp", SRC, *extra]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(verbose=True, extra=sys.argv[1:]))
