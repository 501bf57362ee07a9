#!/bin/bash
# class-64 brain/muscle kernel: bitwise-near comparison with the previous kernel
# (tools/lib_old.so, MPCQP_BM=0), GPU parity subset, config 2/3 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-bm}
MPCQP_LIB=tools/lib_old.so timeout -k 10 120 python tools/lib_compare.py gpurun_out/${T}_old.npz 1024 10 || exit 1
timeout -k 10 120 python tools/lib_compare.py gpurun_out/${T}_new.npz 1024 10 trot10 gpurun_out/${T}_old.npz || exit 1
MPCQP_LIB=tools/lib_old.so timeout -k 10 120 python tools/lib_compare.py gpurun_out/${T}_old3.npz 4096 10 trot10,pace10,bound8 || exit 1
timeout -k 10 120 python tools/lib_compare.py gpurun_out/${T}_new3.npz 4096 10 trot10,pace10,bound8 gpurun_out/${T}_old3.npz || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for c in config2 config3; do
  timeout -k 10 120 python bench.py --no-cpu --no-callers --no-hint-line --config $c --steps 100 --warmup 10 > gpurun_out/${T}_$c.json || exit 1
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], "%.3f MQP/s kernel %.4f ms frac %.3f iters %.1f/%d ok %.4f" % (d["value"]/1e6, d["kernel_ms_avg"], d["roofline"]["frac"], d["iters_mean"], d["iters_max"], d["status_ok_frac"]))' gpurun_out/${T}_$c.json $c
done
for c in "config4 --standing-every 16 --steps 40 --warmup 4" "config5 --standing-every 16 --steps 20 --warmup 2"; do
  name=$(echo $c | cut -d' ' -f1)s16
  timeout -k 10 200 python bench.py --no-cpu --no-callers --no-hint-line --config $c > gpurun_out/${T}_$name.json || exit 1
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], "%.3f MQP/s kernel %.4f ms frac %.3f iters %.1f/%d ok %.4f" % (d["value"]/1e6, d["kernel_ms_avg"], d["roofline"]["frac"], d["iters_mean"], d["iters_max"], d["status_ok_frac"]))' gpurun_out/${T}_$name.json $name
done
