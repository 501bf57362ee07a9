#!/bin/bash
# A/B: config 4 and 5 bench lines (classes 96 / 128) for the in-tree library and variants
#   gpurun -- 'bash tools/gpu_ab45.sh tools/libB.so ...'
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in default "$@"; do
  for c in config4 config5; do
    if [ "$lib" = default ]; then L=""; else L="$lib"; fi
    out=$(MPCQP_LIB=$L timeout -k 10 150 python bench.py --no-cpu --no-callers --config $c --steps 30 --warmup 3) || exit 1
    echo "$lib $c $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.3f MQP/s frac %.3f kernel %.3f ms iters %.1f/%d ok %.3f" % (d["value"]/1e6, d["roofline"]["frac"], d["kernel_ms_avg"], d["iters_mean"], d["iters_max"], d["status_ok_frac"]))')"
  done
done
