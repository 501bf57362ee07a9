#!/bin/bash
# A/B of variant libraries on chosen configs: each argument is LIB:CONFIGS (comma list);
# "default" is the in-tree library.  Parity: each variant's solutions against the in-tree
# ones on every config it is given (tools/lib_compare.py), then REPS rounds of bench lines.
#   gpurun -- 'bash tools/gpu_ab2.sh default:config2,config4 tools/libX.so:config2'
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
REPS=${REPS:-2}
declare -A CARGS=( [config2]="1024 10 trot10" [config3]="4096 10 trot10,pace10,bound8" [config4]="2048 16 trot10,pace10,bound8" [config5]="8192 20 trot10,pace10,bound8" [config4s]="2048 16 trot10,pace10,bound8" )
# config4s: config 4 with every robot standing (the interior-point class); bench only
for spec in "$@"; do
  lib=${spec%%:*}; cfgs=${spec##*:}
  [ "$lib" = default ] && continue
  for c in ${cfgs//,/ }; do
    [ $c = config4s ] && continue
    [ -f gpurun_out/ab_ref_$c.npz ] || { timeout -k 10 150 python tools/lib_compare.py gpurun_out/ab_ref_$c.npz ${CARGS[$c]} || exit 1; }
    echo "== parity $lib $c"
    MPCQP_LIB=$lib timeout -k 10 150 python tools/lib_compare.py gpurun_out/ab_var.npz ${CARGS[$c]} gpurun_out/ab_ref_$c.npz || exit 1
  done
done
for rep in $(seq $REPS); do
for spec in "$@"; do
  lib=${spec%%:*}; cfgs=${spec##*:}
  for c in ${cfgs//,/ }; do
    steps=100; [ $c = config5 ] && steps=30
    cc=$c; extra=""
    [ $c = config4s ] && { cc=config4; extra="--standing-every 1"; steps=8; }
    if [ "$lib" = default ]; then
      out=$(timeout -k 10 180 python bench.py --no-cpu --no-callers --no-hint-line --config $cc $extra --steps $steps --warmup 2) || exit 1
    else
      out=$(MPCQP_LIB=$lib timeout -k 10 180 python bench.py --no-cpu --no-callers --no-hint-line --config $cc $extra --steps $steps --warmup 2) || exit 1
    fi
    echo "$lib $c $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.3f MQP/s kernel %.4f ms frac %.3f iters %.1f/%d ok %.3f" % (d["value"]/1e6, d["kernel_ms_avg"], (d["roofline"]["frac"] or 0), d["iters_mean"], d["iters_max"], d["status_ok_frac"]))')"
  done
done
done
