set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo tests failed; exit 1; }
bash tools/profile.sh r1_v5 > gpurun_out/profile_v5.log 2>&1 || { echo profile failed; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
echo done $?
