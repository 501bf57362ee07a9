#!/bin/bash
# Round 5: interior-point class batched phases on the matrix cores -- IPM parity tests, then an
# A/B of the all-standing config-4 fleet (cold) against variant libraries
#   gpurun -- 'TAG=r5_ipm bash tools/gpu_r5_ipm.sh tools/libA.so ...'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:?set TAG}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 240 --timeout-method thread \
  -k "interior or golden or warm or long_horizon or random_contact or full_weights" > $O/ipm_tests.log 2>&1
rc=$?; tail -3 $O/ipm_tests.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; grep -E "FAIL|Error" $O/ipm_tests.log | head; exit $rc; fi
args=("default:config4s")
for lib in "$@"; do args+=("$lib:config4s"); done
REPS=2 timeout -k 10 600 bash tools/gpu_ab2.sh "${args[@]}" 2>&1 | grep -v amdgpu.ids | tee $O/ab_ipm.txt
