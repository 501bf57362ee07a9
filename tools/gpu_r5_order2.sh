#!/bin/bash
# Round 5: the bucket-sort order kernel -- GPU suite, order 0/1 lines of configs 3-5, the order
# kernel's own time (kernel trace of config 4 / 5), and the solo-vs-shared stamps of config 2
#   gpurun -- 'TAG=r5_order2 bash tools/gpu_r5_order2.sh'
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
  for c in config3 config4 config5; do
    steps=100; [ $c = config5 ] && steps=30
    for o in 0 1; do
      out=$(timeout -k 10 180 python bench.py --no-cpu --no-callers --no-hint-line --config $c --steps $steps --warmup 5 --order $o) || exit 1
      echo "order=$o $c $(echo "$out" | line)" | tee -a $O/ab_order.txt
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for c in config4 config5; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_$c -o kt --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-callers --no-hint-line --config $c --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/$O/kt_$c.json || exit 1
done
cd $GRAFT_REPO_ROOT
grep -h "order_kernel\|kernel_96\|kernel_128" $O/kt_*/kt_kernel_stats.csv | cut -d, -f1-4 | sed 's/((anonymous[^"]*//' | tee $O/order_kernel_time.txt
timeout -k 10 300 python3 tools/solo_stamps.py 1024 > $O/solo_stamps.txt 2>&1 || { tail -5 $O/solo_stamps.txt; exit 1; }
grep -v amdgpu.ids $O/solo_stamps.txt
