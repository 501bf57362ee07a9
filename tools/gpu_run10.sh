#!/bin/bash
# bench (default + the other configs) and the r1_v6 profile
set -o pipefail
mkdir -p gpurun_out/r1_v6
timeout -k 10 300 python bench.py > gpurun_out/r1_v6/bench.json 2> gpurun_out/r1_v6/bench.err || exit 1
for c in config3 config4 config5; do
  timeout -k 10 200 python bench.py --no-cpu --config $c > gpurun_out/r1_v6/bench_$c.json 2>> gpurun_out/r1_v6/bench.err || exit 1
done
bash tools/profile.sh r1_v6 > gpurun_out/r1_v6/profile.log 2>&1 || exit 1
