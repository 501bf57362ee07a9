#!/bin/bash
# Round-5 baseline on a fresh box: GPU suite, the driver's bench command, configs 2-5
#   gpurun -- 'TAG=r5_base bash tools/gpu_r5_base.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:?set TAG}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json || exit $?
timeout -k 10 200 python3 bench.py --no-cpu --no-callers --steps 200 --warmup 20 > $O/bench.json || exit $?
for c in config3 config4 config5; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-callers --config $c > $O/bench_$c.json || exit $?
done
python3 - "$O" <<'PY'
import json, sys, glob, os
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    d = json.load(open(f))
    fr = d.get("roofline") or {}
    print(os.path.basename(f), round(d["value"], 4 if d["unit"] == "ms" else 0), d["unit"],
          "frac", round(fr.get("frac", 0) or 0, 4), "kernel_ms", d.get("kernel_ms_avg"), "iters", d.get("iters_mean"), d.get("iters_max"))
PY
exit $rc
