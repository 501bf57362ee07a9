#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_iter.sh || exit 1
timeout -k 10 200 python bench.py > gpurun_out/bench_default.json || exit 1
cat gpurun_out/bench_default.json
