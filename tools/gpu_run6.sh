set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/pmc_sq.sh c2full > gpurun_out/sq_c2full.txt 2>&1 && \
bash tools/pmc_sq.sh c2it1 --max-iter 1 > gpurun_out/sq_c2it1.txt 2>&1
echo done $?
