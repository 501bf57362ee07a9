#!/bin/bash
# Warm-start check: GPU parity tests of the interior-point class and the drop-in shim,
# then config-1 lines (standing, trot) with warm and cold ticks, and the all-standing
# config-4 fleet (cold: independent batches).
#   gpurun -- 'bash tools/gpu_warm.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/warm
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_shim.py -m gpu -q -x --timeout 200 \
  --timeout-method thread -k "warm or long_horizon or interior or shim or golden" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --config config1 --gait standing --steps 60 --warmup 5 --no-cpu > $O/c1_standing.json || exit $?
timeout -k 10 200 python3 bench.py --config config1 --steps 60 --warmup 5 --no-cpu > $O/c1_trot.json || exit $?
timeout -k 10 200 python3 bench.py --no-cpu --no-callers --no-hint-line --config config4 --standing-every 1 --steps 10 --warmup 2 > $O/c4s.json || exit $?
python3 - <<'PY'
import json
for f in ("c1_standing", "c1_trot", "c4s"):
    d = json.load(open(f"gpurun_out/warm/{f}.json"))
    print(f, d["value"], d["unit"], d.get("iterations_median"), d.get("cold_mpc_tick_ms"))
PY
