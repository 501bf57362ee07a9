#!/bin/bash
# A/B: bench lines of configs 2-5 for the in-tree library and variant libraries, plus a
# bitwise comparison of each variant's config-2 / config-4 solutions against the in-tree one
#   gpurun -- 'bash tools/gpu_ab.sh tools/libA.so tools/libB.so ...'
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CONFIGS=${CONFIGS:-"config2 config3 config4 config5"}
timeout -k 10 120 python tools/lib_compare.py gpurun_out/ab_ref_c2.npz 1024 10 || exit 1
timeout -k 10 120 python tools/lib_compare.py gpurun_out/ab_ref_c4.npz 2048 16 trot10,pace10,bound8 || exit 1
for lib in "$@"; do
  MPCQP_LIB=$lib timeout -k 10 120 python tools/lib_compare.py gpurun_out/ab_var_c2.npz 1024 10 trot10 gpurun_out/ab_ref_c2.npz || exit 1
  MPCQP_LIB=$lib timeout -k 10 120 python tools/lib_compare.py gpurun_out/ab_var_c4.npz 2048 16 trot10,pace10,bound8 gpurun_out/ab_ref_c4.npz || exit 1
done
for rep in 1 2; do
for lib in default "$@"; do
  for c in $CONFIGS; do
    steps=100; [ $c = config5 ] && steps=30
    if [ "$lib" = default ]; then
      out=$(timeout -k 10 180 python bench.py --no-cpu --no-callers --no-hint-line --config $c --steps $steps --warmup 5) || exit 1
    else
      out=$(MPCQP_LIB=$lib timeout -k 10 180 python bench.py --no-cpu --no-callers --no-hint-line --config $c --steps $steps --warmup 5) || exit 1
    fi
    echo "$lib $c $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.3f MQP/s kernel %.4f ms frac %.3f iters %.1f/%d ok %.3f" % (d["value"]/1e6, d["kernel_ms_avg"], (d["roofline"]["frac"] or 0), d["iters_mean"], d["iters_max"], d["status_ok_frac"]))')"
  done
done
done
