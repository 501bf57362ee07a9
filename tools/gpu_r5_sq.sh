#!/bin/bash
# GPU suite, then class-64 SQ counters of config 2 with the active set capped at one
# iteration and uncapped: the difference per iteration is the loop's instruction mix
#   gpurun -- 'TAG=r5_sq bash tools/gpu_r5_sq.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:?set TAG}
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
fi
for cap in 1 0; do
  bash tools/pmc_sq.sh ${TAG}_cap$cap --config config2 --no-hint-line --no-callers --max-iter $cap > $O/sq_cap$cap.txt 2>&1 || { tail -5 $O/sq_cap$cap.txt; exit 1; }
  cp gpurun_out/sq_${TAG}_cap$cap/bench_p1.json $O/bench_cap$cap.json
done
python3 - "$O" <<'PY'
import json, sys, re, os
o = sys.argv[1]
def parse(f):
    d, cur = {}, None
    for line in open(f):
        if not line.startswith(" "):
            cur = line.strip(); continue
        k, v = line.split()[:2]
        if cur == "k64": d[k] = float(v)
    return d
a, b = parse(os.path.join(o, "sq_cap1.txt")), parse(os.path.join(o, "sq_cap0.txt"))
ia = json.load(open(os.path.join(o, "bench_cap1.json")))["iters_mean"]
ib = json.load(open(os.path.join(o, "bench_cap0.json")))["iters_mean"]
w = b["SQ_WAVES"]
print(f"iterations mean cap1 {ia:.2f} uncapped {ib:.2f}; per wave, per iteration (uncapped - cap1):")
for k in sorted(b):
    if k.startswith("SQ_INSTS") or k.startswith("SQ_WAIT") or k.startswith("SQ_ACTIVE") or k == "SQ_WAVE_CYCLES":
        print(f"  {k:28s} cap1 {a[k]/w:10.1f}  full {b[k]/w:10.1f}  per-iter {(b[k]-a[k])/w/(ib-ia):8.1f}")
PY
