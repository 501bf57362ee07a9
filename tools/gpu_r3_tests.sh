#!/bin/bash
# GPU suite + the config-2 bench line (no CPU leg) of the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r3_tests}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 240 python bench.py --no-cpu --no-callers > gpurun_out/${TAG}_c2.json || exit 1
cat gpurun_out/${TAG}_c2.json
