"""Build-level guards (CPU, no GPU needed): the dense QP classes must compile for
gfx950 without private-memory spills.  A spill in the active-set loop costs a
scratch store/load per pass and shows up as HBM write traffic (DESIGN §4.5:
a 4-byte VGPR spill once added ~266 KiB of write-back per config-2 launch)."""
import os
import re
import shutil
import subprocess

import pytest

from mpcqp import build as B

DENSE = ("mpcqp_kernel_64", "mpcqp_kernel_96", "mpcqp_kernel_128")


@pytest.mark.skipif(not os.path.exists(B.HIPCC) and not shutil.which("hipcc"), reason="hipcc not installed")
def test_dense_classes_are_spill_free(tmp_path):
    cmd = [B.HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--cuda-device-only", "-c",
           "-I" + os.path.join(B.ROOT, "include"), "-o", str(tmp_path / "dev.o"), B.SRC,
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, check=True, capture_output=True, text=True).stderr
    usage = {}
    name = None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            usage[name] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+) \[", line)
        if m and name:
            usage[name][m.group(1).strip()] = int(m.group(2))
    for k in DENSE:
        hits = [v for n, v in usage.items() if k in n]
        assert hits, (k, sorted(usage))
        u = hits[0]
        assert u.get("ScratchSize") == 0, (k, u)
        assert u.get("VGPRs Spill") == 0, (k, u)
        assert u.get("Occupancy") >= 2, (k, u)   # two robots' waves per SIMD
