#!/bin/bash
# Round-end GPU pass: full GPU suite, bench lines for configs 2-5, rocprof kernel
# trace + PMC traffic of config 2 (tools/profile.sh).  TAG names the profile set.
#   gpurun -- 'TAG=r1_v10 bash tools/gpu_round.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:?set TAG}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python bench.py > gpurun_out/${TAG}_bench.json || exit 1
for c in config3 config4 config5; do
  timeout -k 10 200 python bench.py --no-cpu --config $c > gpurun_out/${TAG}_bench_$c.json || exit 1
done
bash tools/profile.sh ${TAG} || exit 1
cat gpurun_out/${TAG}_bench.json
