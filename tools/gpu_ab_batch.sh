#!/bin/bash
# A/B across batch sizes: kernel time of config 2 at B = 256 (one robot per CU:
# per-robot latency) .. 4096 (SIMD-shared throughput), default vs variant libraries
#   gpurun -- 'bash tools/gpu_ab_batch.sh tools/libB.so ...'
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in default "$@"; do
  for b in 256 1024 4096; do
    if [ "$lib" = default ]; then L=""; else L="$lib"; fi
    out=$(MPCQP_LIB=$L timeout -k 10 120 python bench.py --no-cpu --no-callers --config config2 --batch $b --steps 60 --warmup 5) || exit 1
    echo "$lib B=$b $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.3f MQP/s kernel %.1f us iters %.1f/%d" % (d["value"]/1e6, d["kernel_ms_avg"]*1e3, d["iters_mean"], d["iters_max"]))')"
  done
done
