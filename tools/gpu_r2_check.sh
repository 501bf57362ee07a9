#!/bin/bash
# Round-2 GPU pass: full GPU suite, default bench line, config-1 drop-in line, the
# interior-point class in configs 4/5 (every 16th robot standing), and the N = 2 path
# spawned by bench.py itself (two ranks on the box's one GPU over gloo).
#   gpurun -- 'TAG=r2_v1 bash tools/gpu_r2_check.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:?set TAG}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json || exit 1
timeout -k 10 300 python bench.py --config config1 --steps 50 --warmup 5 > gpurun_out/${TAG}_bench_config1.json || exit 1
for c in config4 config5; do
  timeout -k 10 300 python bench.py --no-cpu --no-callers --config $c --steps 20 --warmup 3 --standing-every 16 > gpurun_out/${TAG}_bench_${c}_standing16.json || exit 1
done
MPCQP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --no-cpu --no-callers --steps 50 --warmup 5 > gpurun_out/${TAG}_bench_n2_gloo.json || exit 1
cat gpurun_out/${TAG}_bench.json gpurun_out/${TAG}_bench_config1.json
