#!/bin/bash
# Round 5 combined A/B: GPU suite, dispatch order (configs 2-5, --order 0/1), priority variant,
# interior-point phases on the matrix cores (all-standing config 4)
#   gpurun -- 'TAG=r5_combo bash tools/gpu_r5_combo.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:?set TAG}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; grep -E "FAIL|Error" $O/tests.log | head; exit $rc; fi
line() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.3f MQP/s kernel %.4f ms frac %s iters %.1f/%d" % (d["value"]/1e6, d["kernel_ms_avg"], d["roofline"]["frac"], d["iters_mean"], d["iters_max"]))'; }
for rep in 1 2; do
  for c in config2 config3 config4 config5; do
    steps=100; [ $c = config5 ] && steps=30
    for o in 0 1; do
      out=$(timeout -k 10 180 python bench.py --no-cpu --no-callers --no-hint-line --config $c --steps $steps --warmup 5 --order $o) || exit 1
      echo "default order=$o $c $(echo "$out" | line)" | tee -a $O/ab_order.txt
    done
  done
  for c in config2 config3; do
    out=$(MPCQP_LIB=tools/lib_priof1.so timeout -k 10 180 python bench.py --no-cpu --no-callers --no-hint-line --config $c --steps 100 --warmup 5 --order 1) || exit 1
    echo "priof1 order=1 $c $(echo "$out" | line)" | tee -a $O/ab_order.txt
  done
done
REPS=2 timeout -k 10 600 bash tools/gpu_ab2.sh default:config4s tools/lib_ipm_mfma_nowpe.so:config4s tools/lib_ipm_base.so:config4s 2>&1 | grep -v amdgpu.ids | tee $O/ab_ipm.txt
CONFIGS="config2 config3 config4" timeout -k 10 600 bash tools/gpu_ab.sh tools/lib_drop.so 2>&1 | grep -v amdgpu.ids | tee $O/ab_drop.txt
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json || exit $?
echo "driver cmd $(cat $O/bench_driver_cmd.json | line)"
