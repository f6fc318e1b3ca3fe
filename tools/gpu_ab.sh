#!/bin/bash
# A/B session: GPU tests on the in-tree library, then tools/bench_ops.py for the in-tree
# library and every tools/ab/librns_checksum_<name>.so given.  Stops at the first
# timeout / abort / segfault or test failure.
# Usage: bash tools/gpu_ab.sh <tag> "<pytest files>" "<ab names>" [ops] [configs]
set -u
TAG=$1; TESTS=$2; ABS=${3:-}; OPS=${4:-csum,chain,fill,verify}; CFG=${5:-c3_1500B,c5_imix}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$ROOT"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
for v in main $ABS; do
  if [ "$v" = main ]; then L=$ROOT/rustnetworkstack_amd/librns_checksum.so; else L=$ROOT/tools/ab/librns_checksum_$v.so; fi
  RNS_CHECKSUM_LIB=$L timeout -k 10 300 python tools/bench_ops.py --ops "$OPS" --configs "$CFG" --out "$OUT/ops_$v.json" > "$OUT/ops_$v.log" 2>&1
  rc=$?; echo "$v ops rc=$rc"; tail -n 1 "$OUT/ops_$v.log"; [ $rc -eq 0 ] || exit $rc
done
echo "== done"
