#!/bin/bash
# Profile the engine kernel on the GPU box (run from the repo root under gpurun).
#   tools/profile.sh <tag> [bench args...]
# 1. rocprofv3 --kernel-trace --stats   (per-kernel time; must agree with bench.py's HIP events)
# 2. rocprofv3 --pmc FETCH_SIZE          (separate pass, MI355X_MICROARCH.md §HBM)
# 3. rocprofv3 --pmc WRITE_SIZE          (separate pass)
# and writes profiles/<tag>/ (stats CSVs + pmc_traffic.json).
set -euo pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT" "$OUT/summary"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
  python3 bench.py --no-cpu --no-hint-line --steps 20 --warmup 3 "$@" > "$OUT/bench_kt.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o pmc --output-format csv -- \
  python3 bench.py --no-cpu --steps 5 --warmup 1 "$@" > "$OUT/bench_fetch.json"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o pmc --output-format csv -- \
  python3 bench.py --no-cpu --steps 5 --warmup 1 "$@" > "$OUT/bench_write.json"
python3 tools/pmc_summary.py "$OUT" "$OUT/summary" "$@"
