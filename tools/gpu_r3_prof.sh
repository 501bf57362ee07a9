#!/bin/bash
# Round-3 measurements of HEAD: config-1 drop-in lines (trot and STANDING, with the CPU
# port beside them), config-2 phase stamps (stamps build) and SQ counter passes.
#   gpurun -- 'TAG=r3_prof bash tools/gpu_r3_prof.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r3_prof}
timeout -k 10 240 python bench.py --config config1 > gpurun_out/${T}_c1_trot.json || exit 1
tail -1 gpurun_out/${T}_c1_trot.json | cut -c1-400
timeout -k 10 300 python bench.py --config config1 --gait standing --steps 100 --warmup 10 > gpurun_out/${T}_c1_standing.json || exit 1
tail -1 gpurun_out/${T}_c1_standing.json | cut -c1-400
timeout -k 10 120 python tools/phase_stamps.py 1024 10 trot10 > gpurun_out/${T}_stamps_c2.txt 2>&1 || { cat gpurun_out/${T}_stamps_c2.txt; exit 1; }
head -20 gpurun_out/${T}_stamps_c2.txt
bash tools/pmc_sq.sh ${T}_c2 --config config2 > gpurun_out/${T}_sq_c2.txt 2>&1 || { tail -20 gpurun_out/${T}_sq_c2.txt; exit 1; }
cat gpurun_out/${T}_sq_c2.txt
