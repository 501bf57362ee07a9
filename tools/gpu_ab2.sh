#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
ALT=${1:-pympc-quadruped_amd/mpcqp/libmpcqp_nopair.so}
for b in 256 512 1024; do
  timeout -k 10 120 python bench.py --no-cpu --no-callers --batch $b > gpurun_out/ab2_A_$b.json || exit 1
  MPCQP_LIB=$ALT timeout -k 10 120 python bench.py --no-cpu --no-callers --batch $b > gpurun_out/ab2_B_$b.json || exit 1
done
python - <<'PY'
import json
for b in (256, 512, 1024):
    for v in ("A", "B"):
        d = json.load(open(f"gpurun_out/ab2_{v}_{b}.json"))
        print(b, v, round(d["kernel_ms_avg"] * 1e3, 1), "us iters", round(d["iters_mean"], 2), d["iters_max"])
PY
