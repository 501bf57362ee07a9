#!/bin/bash
# A/B of the interior-point class: standing robots (tools/ipm_stats.py: B = 1 and B = 256
# latency, factorisations, parity) for the in-tree library and variant libraries
#   gpurun -- 'bash tools/ipm_ab.sh tools/libB.so ...'
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in default "$@"; do
  if [ "$lib" = default ]; then L=""; else L="$lib"; fi
  echo "== $lib"
  MPCQP_LIB=$L B=1 timeout -k 10 120 python tools/ipm_stats.py 2>&1 | grep standing || exit 1
  MPCQP_LIB=$L B=256 PARITY=1 timeout -k 10 120 python tools/ipm_stats.py 2>&1 | grep -E "standing|parity" || exit 1
done
