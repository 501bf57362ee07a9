#!/bin/bash
# Interior-point layout choice per launch (throughput layout for a large direct batch,
# latency layout otherwise) and the bench's exact stance range: IPM/shim parity tests, then
# the lines it touches.
#   gpurun -- 'bash tools/gpu_layout.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/layout
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_shim.py -m gpu -q -x --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --no-cpu --no-callers > $O/c2.json || exit $?
for c in config3 config4 config5; do timeout -k 10 200 python3 bench.py --no-cpu --no-callers --config $c > $O/$c.json || exit $?; done
timeout -k 10 200 python3 bench.py --no-cpu --no-callers --no-hint-line --config config4 --standing-every 1 --steps 10 --warmup 2 > $O/c4s.json || exit $?
timeout -k 10 200 python3 bench.py --no-cpu --no-callers --config config4 --standing-every 16 --steps 40 --warmup 4 > $O/c4s16.json || exit $?
timeout -k 10 200 python3 bench.py --config config1 --gait standing --steps 40 --warmup 5 --no-cpu > $O/c1s.json || exit $?
python3 - <<'PY'
import json
for f in ("c2", "config3", "config4", "config5", "c4s", "c4s16", "c1s"):
    d = json.load(open(f"gpurun_out/layout/{f}.json"))
    print(f, round(d["value"], 4 if d["unit"] == "ms" else 0), d["unit"], d.get("stance_range"), (d.get("no_hint") or {}).get("value"),
          (d.get("cold_mpc_tick_ms") or {}).get("median"))
PY
