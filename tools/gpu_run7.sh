set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in config3 config4 config5; do
  timeout -k 10 200 python bench.py --no-cpu --config $c > gpurun_out/bench_$c.json 2>/dev/null || exit 1
done
timeout -k 10 120 python tools/phase_stamps.py 2048 16 trot10,pace10,bound8 > gpurun_out/stamps_c4.txt 2>&1
echo done $?
