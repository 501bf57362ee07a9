#!/bin/bash
# A/B: config 2 and 3 bench lines for the in-tree library and variant libraries
#   gpurun -- 'bash tools/gpu_ab.sh tools/libA.so tools/libB.so ...'
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in default "$@"; do
  for c in config2 config3; do
    if [ "$lib" = default ]; then
      out=$(timeout -k 10 120 python bench.py --no-cpu --no-callers --config $c --steps 100 --warmup 10) || exit 1
    else
      out=$(MPCQP_LIB=$lib timeout -k 10 120 python bench.py --no-cpu --no-callers --config $c --steps 100 --warmup 10) || exit 1
    fi
    echo "$lib $c $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.3f MQP/s frac %.3f iters %.1f/%d ok %.3f" % (d["value"]/1e6, d["roofline"]["frac"], d["iters_mean"], d["iters_max"], d["status_ok_frac"]))')"
  done
done
