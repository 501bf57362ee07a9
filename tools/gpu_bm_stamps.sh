#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-bms}
timeout -k 10 120 python tools/bm_stamps.py 1024 10 > gpurun_out/${T}_c2.txt 2>&1 && \
timeout -k 10 120 python tools/bm_stamps.py 256 10 > gpurun_out/${T}_b256.txt 2>&1
rc=$?
cat gpurun_out/${T}_c2.txt gpurun_out/${T}_b256.txt
exit $rc
