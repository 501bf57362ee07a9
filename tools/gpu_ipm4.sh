#!/bin/bash
# Interior-point class at four robots per CU (N <= 16: M_k in the global slot): IPM parity
# tests, then the A/B against the three-per-CU build on the standing lines.
#   gpurun -- 'bash tools/gpu_ipm4.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ipm4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_shim.py -m gpu -q -x --timeout 200 \
  --timeout-method thread -k "warm or long_horizon or interior or shim or golden or random_contact or standing or eviction" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for lib in default tools/lib_ipm3cu.so; do
  for rep in 1 2; do
    if [ $lib = default ]; then E=""; else E="MPCQP_LIB=$lib"; fi
    env $E timeout -k 10 200 python3 bench.py --no-cpu --no-callers --no-hint-line --config config4 --standing-every 1 --steps 10 --warmup 2 > $O/c4s_$rep.json || exit $?
    env $E timeout -k 10 200 python3 bench.py --no-cpu --no-callers --no-hint-line --config config4 --standing-every 1 --warm-fleet --steps 12 --warmup 2 > $O/c4sw_$rep.json || exit $?
    env $E timeout -k 10 200 python3 bench.py --config config1 --gait standing --steps 40 --warmup 5 --no-cpu > $O/c1s_$rep.json || exit $?
    python3 - "$lib" "$O" "$rep" <<'PY'
import json, sys
lib, o, rep = sys.argv[1:]
a = json.load(open(f"{o}/c4s_{rep}.json")); w = json.load(open(f"{o}/c4sw_{rep}.json")); c = json.load(open(f"{o}/c1s_{rep}.json"))
print(lib, "cold fleet %.3f MQP/s" % (a["value"] / 1e6), "warm fleet %.3f MQP/s" % (w["value"] / 1e6),
      "c1 standing warm %.3f ms cold %.3f ms" % (c["value"], c["cold_mpc_tick_ms"]["median"]))
PY
  done
done
