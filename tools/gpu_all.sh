#!/bin/bash
# GPU tests + smoke once, then for every BASELINE.json GPU config: the driver's bench
# command under rocprofv3 --kernel-trace --stats (reconciled) and the PMC traffic passes.
# Usage: bash tools/gpu_all.sh <tag> [configs...]
set -u
TAG=${1:-r02}; shift
CONFIGS=${@:-c3_1500B c2_64B c4_9000B c5_imix}
bash tools/gpu_session.sh ${TAG}_tests c3_1500B 20 5 || exit $?
for c in $CONFIGS; do
  [ "$c" = c3_1500B ] && continue
  K=20; [ "$c" = c2_64B ] && K=200   # ~13 us steps: amortise the graph launch over more of them
  SKIP_TESTS=1 bash tools/gpu_session.sh ${TAG}_$c $c $K 5 || exit $?
done
