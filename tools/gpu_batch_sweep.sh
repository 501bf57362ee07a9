#!/bin/bash
# kernel time vs batch at config2 (SIMD sharing vs per-robot latency)
set -o pipefail
mkdir -p gpurun_out
for b in 256 512 1024 2048; do
  timeout -k 10 120 python bench.py --no-cpu --no-callers --config config2 --batch $b > gpurun_out/bs_$b.json || exit 1
done
python - <<'PY'
import json
for b in (256, 512, 1024, 2048):
    d = json.load(open(f"gpurun_out/bs_{b}.json"))
    print(b, round(d["value"]), "QP/s", round(d["kernel_ms_avg"]*1e3, 1), "us", "iters", round(d["iters_mean"], 2), d["iters_max"], "us/maxiter", round(d["kernel_ms_avg"]*1e3/d["iters_max"], 2))
PY
