set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && \
timeout -k 10 200 python bench.py --no-cpu --config config3 > gpurun_out/bench_c3.json 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --config config4 > gpurun_out/bench_c4.json 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --config config5 > gpurun_out/bench_c5.json 2>&1 && \
timeout -k 10 120 python tools/phase_stamps.py 1024 10 > gpurun_out/stamps_c2.txt 2>&1 && \
timeout -k 10 120 python tools/phase_stamps.py 2048 16 trot10,pace10,bound8 > gpurun_out/stamps_c4.txt 2>&1
echo done $?
