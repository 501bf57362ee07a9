#!/bin/bash
# Round-6 profile set (TAG names it): GPU suite, the driver's bench command, bench lines of
# configs 2-5 (+ the batch-order sub-line), the standing fleets and config 1.  PART=2: rocprof
# kernel trace + PMC traffic of configs 2-5 (tools/profile.sh: profiles/<tag>/pmc_traffic.json
# keyed by this build's SHA-256), phase stamps of classes 64 / 96 / 128, SQ counters of configs
# 4 and 5.  A test failure does not stop the bench lines; a timeout, crash or abort ends it.
#   gpurun -- 'TAG=r6_final bash tools/gpu_r6_final.sh'; gpurun -- 'TAG=r6_final PART=2 bash tools/gpu_r6_final.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:?set TAG}
O=gpurun_out/$TAG
mkdir -p $O
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json || exit $?
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 > $O/bench.json || exit $?
timeout -k 10 200 python3 bench.py --no-cpu --no-callers --no-hint-line --steps 200 --warmup 20 --order 0 > $O/bench_order0.json || exit $?
for c in config3 config4 config5; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-callers --config $c > $O/bench_$c.json || exit $?
  timeout -k 10 200 python3 bench.py --no-cpu --no-callers --no-hint-line --config $c --order 0 > $O/bench_${c}_order0.json || exit $?
done
timeout -k 10 200 python3 bench.py --no-cpu --no-callers --no-hint-line --config config4 --standing-every 1 --steps 10 --warmup 2 > $O/bench_config4_standing1.json || exit $?
timeout -k 10 200 python3 bench.py --no-cpu --no-callers --no-hint-line --config config4 --standing-every 1 --cross-leg-r --steps 6 --warmup 1 > $O/bench_config4_standing1_crossR.json || exit $?
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
          "frac", fr.get("frac"), "kernel_ms", d.get("kernel_ms_avg"), "iters", d.get("iters_mean"), d.get("iters_max"))
PY
else
for c in config2 config3 config4 config5; do
  bash tools/profile.sh $TAG --config $c > $O/profile_$c.log 2>&1 || { tail -20 $O/profile_$c.log; exit 1; }
  cp gpurun_out/prof_$TAG/summary/kt_kernel_stats.csv $O/kt_${c}_kernel_stats.csv
  cp gpurun_out/prof_$TAG/bench_kt.json $O/bench_kt_$c.json
done
[ -n "$PROFILE_ONLY" ] && { echo done; exit 0; }
timeout -k 10 150 python3 tools/phase_stamps.py 1024 10 trot10 > $O/stamps_c2.txt 2>&1 || exit $?
timeout -k 10 200 python3 tools/phase_stamps.py 2048 16 trot10,pace10,bound8 > $O/stamps_c4_class96.txt 2>&1 || exit $?
timeout -k 10 300 python3 tools/phase_stamps.py 8192 20 trot10,pace10,bound8 > $O/stamps_c5_class128.txt 2>&1 || exit $?
bash tools/pmc_sq.sh ${TAG}_c2 --config config2 --no-hint-line > $O/sq_c2_class64.txt 2>&1 || { tail -5 $O/sq_c2_class64.txt; exit 1; }
bash tools/pmc_sq.sh ${TAG}_c4 --config config4 --no-hint-line > $O/sq_c4_class96.txt 2>&1 || { tail -5 $O/sq_c4_class96.txt; exit 1; }
bash tools/pmc_sq.sh ${TAG}_c5 --config config5 --no-hint-line > $O/sq_c5_class128.txt 2>&1 || { tail -5 $O/sq_c5_class128.txt; exit 1; }
echo done
fi
