set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/phase_stamps.py 1024 10 > gpurun_out/r2_stamps_c2.txt 2>&1 && \
timeout -k 10 120 python tools/phase_stamps.py 4096 10 trot10,pace10,bound8 > gpurun_out/r2_stamps_c3.txt 2>&1 && \
bash tools/pmc_sq.sh r2_v1 > gpurun_out/r2_sq_summary.txt 2>&1
rc=$?
cat gpurun_out/r2_stamps_c2.txt gpurun_out/r2_sq_summary.txt
exit $rc
