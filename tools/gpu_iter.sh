#!/bin/bash
# Iteration check: GPU parity suite, bench lines for configs 2-5, phase stamps (configs 2-4).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_quick.sh || exit 1
timeout -k 10 120 python tools/phase_stamps.py 1024 10 > gpurun_out/stamps_c2.txt 2>&1 || exit 1
timeout -k 10 120 python tools/phase_stamps.py 4096 10 trot10,pace10,bound8 > gpurun_out/stamps_c3.txt 2>&1 || exit 1
timeout -k 10 120 python tools/phase_stamps.py 2048 16 trot10,pace10,bound8 > gpurun_out/stamps_c4.txt 2>&1 || exit 1
head -9 gpurun_out/stamps_c2.txt; head -9 gpurun_out/stamps_c4.txt; tail -8 gpurun_out/stamps_c4.txt
