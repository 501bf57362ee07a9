#!/bin/bash
# class 96 (config 4): phase stamps (stamps build) and SQ counter passes of HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r3c96}
timeout -k 10 120 python tools/phase_stamps.py 2048 16 trot10,pace10,bound8 > gpurun_out/${T}_stamps_c4.txt 2>&1 || { cat gpurun_out/${T}_stamps_c4.txt; exit 1; }
head -12 gpurun_out/${T}_stamps_c4.txt
bash tools/pmc_sq.sh ${T}_c4 --config config4 > gpurun_out/${T}_sq_c4.txt 2>&1 || { tail -20 gpurun_out/${T}_sq_c4.txt; exit 1; }
cat gpurun_out/${T}_sq_c4.txt
