"""GPU: bench.py's single-GPU path end to end (one JSON line, the contract fields)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_bench_contract_line():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                          "--cpu-seconds", "0.5"], capture_output=True, text=True, timeout=600, check=True)
    line = json.loads(out.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["value"] > 0 and line["n_gpus"] == 1 and line["scaling"] == "weak"
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(line["roofline"])
    assert line["roofline"]["bound"] == "valu"   # FP64 vector pipe: no MFMA on the path
    cpu = line["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["cores"] >= 1 and cpu["value"] > 0
    assert cpu["single_core"]["cores"] == 1 and cpu["single_core"]["value"] > 0
    assert line["status_ok_frac"] == 1.0


def test_bench_config1_drop_in_latency():
    """Config 1: the drop-in controller's per-tick latency line (B = 1, horizon 16)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "config1", "--steps", "5",
                          "--warmup", "2", "--cpu-seconds", "0.5"], capture_output=True, text=True, timeout=600,
                         check=True)
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["higher_is_better"] is False and line["unit"] == "ms" and line["value"] > 0
    assert line["config"]["horizon"] == 16 and line["cpu_baseline"]["value"] > 0
