#!/bin/bash
# Round-4 GPU check: the GPU suite, the driver's bench command, and optional extra bench
# lines.  A test failure (pytest rc 1) does not stop the bench lines; a timeout, crash or
# abort (any other non-zero rc) ends the script there.
#   gpurun -- 'TAG=r4a EXTRA="--config config4 --standing-every 1 --steps 5 --warmup 1" bash tools/gpu_r4.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:?set TAG}
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread ${PYTEST_ARGS} > $O/tests.log 2>&1
  rc=$?
  tail -3 $O/tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
fi
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.json || exit $?
python -c "import json; d=json.load(open('$O/bench.json')); print('config2', round(d['value']), 'QP/s', round(d['kernel_ms_avg'],4), 'ms frac', round(d['roofline']['frac'],4), 'iters', round(d['iters_mean'],2), d['iters_max'])"
i=0
while IFS= read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu --no-callers $line > $O/extra_$i.json || exit $?
  python -c "import json; d=json.load(open('$O/extra_$i.json')); print('$line |', round(d['value']), 'QP/s', round(d['kernel_ms_avg'],4), 'ms frac', round(d['roofline']['frac'],4) if d.get('roofline') else None, 'iters', round(d.get('iters_mean',0),2), d.get('iters_max'))"
done <<< "$EXTRA"
echo done
