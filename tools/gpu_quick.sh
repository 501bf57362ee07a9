#!/bin/bash
# quick GPU check: parity tests + config2/config3 bench lines (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
timeout -k 10 200 python bench.py --no-cpu --no-callers > gpurun_out/q_c2.json || exit 1
timeout -k 10 200 python bench.py --no-cpu --no-callers --config config3 > gpurun_out/q_c3.json || exit 1
python - <<'PY'
import json
for c in ("c2", "c3"):
    d = json.load(open(f"gpurun_out/q_{c}.json"))
    print(c, round(d["value"]), "QP/s", round(d["kernel_ms_avg"], 4), "ms", round(d["roofline"]["frac"], 4), "iters", d["iters_mean"], d["iters_max"])
PY
