#!/bin/bash
# quick GPU check: parity tests + bench lines for configs 2-5 (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
for c in config2 config3 config4 config5; do
  timeout -k 10 200 python bench.py --no-cpu --no-callers --config $c > gpurun_out/q_$c.json || exit 1
done
python - <<'PY'
import json
for c in ("config2", "config3", "config4", "config5"):
    d = json.load(open(f"gpurun_out/q_{c}.json"))
    print(c, round(d["value"]), "QP/s", round(d["kernel_ms_avg"], 4), "ms", round(d["roofline"]["frac"], 4), "iters", round(d["iters_mean"], 2), d["iters_max"])
PY
