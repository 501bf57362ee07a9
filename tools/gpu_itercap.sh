#!/bin/bash
# kernel time vs active-set iteration cap (B = 256: one robot per CU; B = 1024):
# the slope is the uninstrumented cost of one iteration of the slowest robots
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 256 1024; do
  for cap in 1 10 20 30 40 50 60 80; do
    out=$(timeout -k 10 120 python bench.py --no-cpu --no-callers --config config2 --batch $b --steps 40 --warmup 5 --max-iter $cap) || exit 1
    echo "B=$b cap=$cap $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("kernel %.1f us iters %.1f/%d" % (d["kernel_ms_avg"]*1e3, d["iters_mean"], d["iters_max"]))')"
  done
done
