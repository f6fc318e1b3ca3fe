#!/bin/bash
# A/B session on the packed form: GPU tests on the in-tree library, then
# tools/probe_packed_ab.py alternating the in-tree library and every
# tools/ab/librns_checksum_<name>.so given, REPS times (drift shows as main/main spread).
# Stops at the first timeout / abort / segfault or test failure.
# CHAINS=<configs> also times rns_csum_chain_dev (tools/bench_ops.py --ops chain).
# Usage: bash tools/gpu_abp.sh <tag> "<pytest files>" "<ab names>" [reps] [configs]
set -u
TAG=$1; TESTS=$2; ABS=${3:-}; REPS=${4:-2}; CFG=${5:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$ROOT"
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq 1 "$REPS"); do
  for v in main $ABS; do
    if [ "$v" = main ]; then L=$ROOT/rustnetworkstack_amd/librns_checksum.so; else L=$ROOT/tools/ab/librns_checksum_$v.so; fi
    EXTRA=""; [ -n "$CFG" ] && EXTRA="--configs $CFG"
    RNS_CHECKSUM_LIB=$L timeout -k 10 300 python tools/probe_packed_ab.py --label "$v" $EXTRA --out "$OUT/abp_${v}_$rep.json" > "$OUT/abp_${v}_$rep.log" 2>&1
    rc=$?; echo "$v rep $rep rc=$rc"; grep -v '^{' "$OUT/abp_${v}_$rep.log" | tail -n 8; [ $rc -eq 0 ] || exit $rc
    if [ -n "${CHAINS:-}" ]; then  # fragment chains (packed [492, 512, rest] and NetBuffer layouts)
      RNS_CHECKSUM_LIB=$L timeout -k 10 300 python tools/bench_ops.py --ops chain --configs "$CHAINS" --out "$OUT/chain_${v}_$rep.json" > "$OUT/chain_${v}_$rep.log" 2>&1
      rc=$?; echo "$v chains rc=$rc"; grep -v '^{' "$OUT/chain_${v}_$rep.log" | tail -n 3; [ $rc -eq 0 ] || exit $rc
    fi
  done
done
echo "== done"
