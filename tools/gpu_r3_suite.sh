#!/bin/bash
# full GPU suite + bench lines for configs 2-5 and the standing mixes (no CPU leg)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r3s}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
run() {
  local name=$1; shift
  timeout -k 10 240 python bench.py --no-cpu --no-callers "$@" > gpurun_out/${T}_$name.json || { echo "FAIL $name"; exit 1; }
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); nh=d.get("no_hint") or {}; ts=d.get("two_streams") or {}; print(sys.argv[2], "%.3f MQP/s kernel %.4f ms frac %.3f iters %.1f/%d ok %.4f no_hint %.3f two_streams %.3f" % (d["value"]/1e6, d["kernel_ms_avg"], d["roofline"]["frac"], d["iters_mean"], d["iters_max"], d["status_ok_frac"], nh.get("value", 0)/1e6, ts.get("value", 0)/1e6))' gpurun_out/${T}_$name.json $name
}
run c2 --config config2
run c3 --config config3
run c4 --config config4
run c5 --config config5 --steps 60 --warmup 5
run c4s16 --config config4 --standing-every 16 --steps 40 --warmup 4
run c5s16 --config config5 --standing-every 16 --steps 20 --warmup 2
