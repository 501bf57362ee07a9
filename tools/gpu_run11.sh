set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/phase_stamps.py 1024 10 > gpurun_out/stamps_c2.txt 2>&1 && \
timeout -k 10 120 python tools/phase_stamps.py 64 10 > gpurun_out/stamps_b64.txt 2>&1
echo done $?
