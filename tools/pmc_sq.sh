#!/bin/bash
# SQ counter passes (separate --pmc runs, kernel-trace only) for the engine kernels.
#   tools/pmc_sq.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:?tag}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/sq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $SET -d "$OUT/p$i" -o pmc --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 5 --warmup 1 "$@" > "$OUT/bench_p$i.json"
done
python3 $GRAFT_REPO_ROOT/tools/sq_summary.py "$OUT"
