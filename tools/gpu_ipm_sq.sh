#!/bin/bash
# SQ counters of the interior-point class on the all-standing config-4 fleet (cold), plus
# the instruction-cache counters this box exposes.
#   gpurun -- 'bash tools/gpu_ipm_sq.sh'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ipm_sq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/$O/counters.txt 2>&1 || true
grep -i -E "SQC|ICACHE|IFETCH|INST_LEVEL|WAIT_INST" $GRAFT_REPO_ROOT/$O/counters.txt | head -40 > $GRAFT_REPO_ROOT/$O/icache_counters.txt || true
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $SET -d $GRAFT_REPO_ROOT/$O/p$i -o pmc --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-callers --no-hint-line --config config4 --standing-every 1 --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/bench_p$i.json || exit $?
done
cat $GRAFT_REPO_ROOT/$O/icache_counters.txt | head -30
