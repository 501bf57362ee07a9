#!/bin/bash
# A/B: the in-tree build vs an alternative library (MPCQP_LIB), configs 2 and 3, interleaved
set -o pipefail
mkdir -p gpurun_out
ALT=${1:-pympc-quadruped_amd/mpcqp/libmpcqp_nopair.so}
for rep in 1 2; do
  for c in config2 config3; do
    timeout -k 10 120 python bench.py --no-cpu --no-callers --config $c > gpurun_out/ab_A_${c}_$rep.json || exit 1
    MPCQP_LIB=$ALT timeout -k 10 120 python bench.py --no-cpu --no-callers --config $c > gpurun_out/ab_B_${c}_$rep.json || exit 1
  done
done
python - <<'PY'
import json
for c in ("config2", "config3"):
    for v in ("A", "B"):
        r = [json.load(open(f"gpurun_out/ab_{v}_{c}_{k}.json")) for k in (1, 2)]
        print(c, v, [round(d["kernel_ms_avg"] * 1e3, 1) for d in r], "us", "iters", r[0]["iters_mean"], r[0]["iters_max"])
PY
