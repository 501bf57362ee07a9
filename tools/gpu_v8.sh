#!/bin/bash
# Round-1 re-entry: full GPU suite, bench lines for configs 2-5, rocprof profile of config 2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/v8_tests.log 2>&1 || { tail -30 gpurun_out/v8_tests.log; exit 1; }
tail -1 gpurun_out/v8_tests.log
timeout -k 10 200 python bench.py > gpurun_out/v8_bench.json || exit 1
for c in config3 config4 config5; do
  timeout -k 10 200 python bench.py --no-cpu --config $c > gpurun_out/v8_bench_$c.json || exit 1
done
bash tools/profile.sh r1_v8 || exit 1
cat gpurun_out/v8_bench.json
