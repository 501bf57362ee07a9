#!/bin/bash
# ablation timing: kernel time at an iteration cap for the in-tree library and variants
#   gpurun -- 'bash tools/gpu_abl.sh tools/libA.so ...'
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in default "$@"; do
  for b in ${BATCHES:-256 1024}; do
    for cap in ${CAPS:-1 20 40}; do
      if [ "$lib" = default ]; then L=""; else L="MPCQP_LIB=$lib"; fi
      out=$(env $L timeout -k 10 120 python bench.py --no-cpu --no-callers --no-hint-line --config config2 --batch $b --steps 40 --warmup 5 --max-iter $cap) || exit 1
      echo "$lib B=$b cap=$cap $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("kernel %.1f us iters %.1f/%d" % (d["kernel_ms_avg"]*1e3, d["iters_mean"], d["iters_max"]))')"
    done
  done
done
