#!/bin/bash
# Config 1 (drop-in, B = 1): shim GPU tests, the bench line, and a rocprofv3 kernel +
# memory-copy trace of the same loop (per-tick kernel / copy durations).
#   gpurun -- 'TAG=r2_c1 bash tools/gpu_c1.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-c1}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_shim.py tests/test_gpu_dist.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python bench.py --config config1 > gpurun_out/${TAG}_bench.json || exit 1
cat gpurun_out/${TAG}_bench.json
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT -o c1 --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --config config1 --steps 60 --warmup 10 --cpu-seconds 0.5 \
  > $OUT.json 2>&1 || exit 1
cat $OUT/c1_kernel_stats.csv
