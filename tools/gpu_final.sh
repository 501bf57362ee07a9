#!/bin/bash
# Round-end profile set: gpu_round.sh (GPU suite, bench lines configs 2-5, rocprof kernel
# trace + PMC traffic of config 2), then the standing mixes and the config-1 drop-in lines.
#   gpurun -- 'TAG=r3_s2f bash tools/gpu_final.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:?set TAG}
mkdir -p gpurun_out
bash tools/gpu_round.sh > gpurun_out/${TAG}_round.txt 2>&1 || { tail -30 gpurun_out/${TAG}_round.txt; exit 1; }
timeout -k 10 240 python bench.py --no-cpu --no-callers --config config4 --standing-every 16 --steps 40 --warmup 4 > gpurun_out/${TAG}_bench_c4s16.json || exit 1
timeout -k 10 300 python bench.py --no-cpu --no-callers --config config5 --standing-every 16 --steps 20 --warmup 2 > gpurun_out/${TAG}_bench_c5s16.json || exit 1
timeout -k 10 240 python bench.py --config config1 > gpurun_out/${TAG}_c1_trot.json || exit 1
timeout -k 10 300 python bench.py --config config1 --gait standing --steps 100 --warmup 10 > gpurun_out/${TAG}_c1_standing.json || exit 1
timeout -k 10 120 python tools/phase_stamps.py 1024 10 trot10 > gpurun_out/${TAG}_stamps_c2.txt 2>&1 || exit 1
echo done
