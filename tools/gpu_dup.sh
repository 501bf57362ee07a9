#!/bin/bash
# price loop components on the critical path: bench lines of duplicate-component builds
# (same decisions, same results) against the in-tree library
#   gpurun -- 'bash tools/gpu_dup.sh tools/lib_dup1.so ...'
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for lib in default "$@"; do
  for c in ${CONFIGS:-config2}; do
    if [ "$lib" = default ]; then L=""; else L="MPCQP_LIB=$lib"; fi
    for b in ${BATCHES:-1024 256}; do
      out=$(env $L timeout -k 10 120 python bench.py --no-cpu --no-callers --no-hint-line --config $c --batch $b --steps 100 --warmup 5) || exit 1
      echo "$lib $c B=$b $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.3f MQP/s kernel %.2f us iters %.1f/%d" % (d["value"]/1e6, d["kernel_ms_avg"]*1e3, d["iters_mean"], d["iters_max"]))')"
    done
  done
done
done
