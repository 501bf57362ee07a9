#!/bin/bash
# Round-6 A/B: the first library is the reference.  Each other library's solutions are compared
# with it (configs 2 / 4 / 5 shapes: classes 64 / 96 / 128), then bench lines of $CONFIGS for every
# library, two interleaved repetitions; SQ=1 adds one LDS-counter pass per library on config 5
# (class 128) and config 2 (class 64).  TESTS=1 runs the GPU suite (in-tree library) first.
#   gpurun -- 'TESTS=1 SQ=1 bash tools/gpu_r6_ab.sh tools/lib_base.so tools/lib_x.so'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r6ab}
mkdir -p $O
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log
  [ $rc -ne 0 ] && { echo "pytest rc $rc: stopping"; exit $rc; }
fi
REF=$1
MPCQP_LIB=$REF timeout -k 10 120 python tools/lib_compare.py $O/ref_c2.npz 1024 10 || exit 1
MPCQP_LIB=$REF timeout -k 10 120 python tools/lib_compare.py $O/ref_c4.npz 2048 16 trot10,pace10,bound8 || exit 1
MPCQP_LIB=$REF timeout -k 10 120 python tools/lib_compare.py $O/ref_c5.npz 2048 20 trot10,pace10,bound8 || exit 1
for lib in "${@:2}"; do
  echo "== $lib vs $REF"
  MPCQP_LIB=$lib timeout -k 10 120 python tools/lib_compare.py $O/var_c2.npz 1024 10 trot10 $O/ref_c2.npz || exit 1
  MPCQP_LIB=$lib timeout -k 10 120 python tools/lib_compare.py $O/var_c4.npz 2048 16 trot10,pace10,bound8 $O/ref_c4.npz || exit 1
  MPCQP_LIB=$lib timeout -k 10 120 python tools/lib_compare.py $O/var_c5.npz 2048 20 trot10,pace10,bound8 $O/ref_c5.npz || exit 1
done
CONFIGS=${CONFIGS:-"config2 config4 config5"}
for rep in 1 2; do
for lib in "$@"; do
  for c in $CONFIGS; do
    steps=100; [ $c = config5 ] && steps=30
    out=$(MPCQP_LIB=$lib timeout -k 10 180 python bench.py --no-cpu --no-callers --no-hint-line --config $c --steps $steps --warmup 5) || exit 1
    echo "$lib $c $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.3f MQP/s kernel %.4f ms frac %.3f iters %.1f/%d ok %.3f" % (d["value"]/1e6, d["kernel_ms_avg"], (d["roofline"]["frac"] or 0), d["iters_mean"], d["iters_max"], d["status_ok_frac"]))')"
  done
done
done
if [ "${SQ:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  SET="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU"
  i=0
  for lib in "$@"; do
    i=$((i+1))
    for c in config5 config2; do
      d=$GRAFT_REPO_ROOT/$O/sq_${i}_$c
      MPCQP_LIB=$GRAFT_REPO_ROOT/$lib timeout -s KILL 120 rocprofv3 --pmc $SET -d $d -o pmc --output-format csv -- \
        python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-callers --no-hint-line --steps 5 --warmup 1 --config $c > $d.json 2> $d.err || { tail -5 $d.err; exit 1; }
      echo "== SQ $lib $c"
      python3 $GRAFT_REPO_ROOT/tools/sq_summary.py $d | grep -A9 -E "^k(64|128)"
    done
  done
fi
echo done
