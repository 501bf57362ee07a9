#!/bin/bash
# Round-4 profile set (TAG names it): GPU suite, the driver's bench command, bench lines of
# configs 3-5, the standing fleets and config 1, rocprof kernel trace + PMC traffic of
# config 2 (tools/profile.sh: profiles/latest/pmc_traffic.json is keyed by this build's
# SHA-256), phase stamps.  A test failure does not stop the bench lines; a timeout, crash or
# abort ends the script.
#   gpurun -- 'TAG=r4_final bash tools/gpu_r4_final.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:?set TAG}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json || exit $?
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 > $O/bench.json || exit $?
for c in config3 config4 config5; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-callers --config $c > $O/bench_$c.json || exit $?
done
timeout -k 10 200 python3 bench.py --no-cpu --no-callers --no-hint-line --config config4 --standing-every 1 --steps 10 --warmup 2 > $O/bench_config4_standing1.json || exit $?
timeout -k 10 200 python3 bench.py --no-cpu --no-callers --no-hint-line --config config4 --standing-every 1 --warm-fleet --steps 12 --warmup 2 > $O/bench_config4_standing1_warm.json || exit $?
timeout -k 10 200 python3 bench.py --no-cpu --no-callers --config config4 --standing-every 16 --steps 40 --warmup 4 > $O/bench_config4_standing16.json || exit $?
timeout -k 10 300 python3 bench.py --no-cpu --no-callers --config config5 --standing-every 16 --steps 20 --warmup 2 > $O/bench_config5_standing16.json || exit $?
timeout -k 10 200 python3 bench.py --config config1 --cpu-seconds 4 > $O/c1_trot.json || exit $?
timeout -k 10 200 python3 bench.py --config config1 --gait standing --steps 100 --warmup 10 --cpu-seconds 4 > $O/c1_standing.json || exit $?
python3 - "$O" <<'PY'
import json, sys, glob, os
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    d = json.load(open(f))
    fr = d.get("roofline") or {}
    print(os.path.basename(f), round(d["value"], 4 if d["unit"] == "ms" else 0), d["unit"],
          "frac", round(fr.get("frac", 0) or 0, 4), "iters", d.get("iters_mean"), d.get("iters_max"))
PY
bash tools/profile.sh $TAG > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
timeout -k 10 150 python3 tools/phase_stamps.py 1024 10 trot10 > $O/stamps_c2.txt 2>&1 || exit $?
echo done
