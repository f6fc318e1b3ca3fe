#!/bin/bash
# A/B of library builds on the widened ops (tools/bench_ops.py) and bench.py --op verify,
# alternating builds, REPS times.  Usage: bash tools/ops_ab.sh <tag> "<ab names>" [reps] [ops] [configs]
set -u
TAG=$1; ABS=$2; REPS=${3:-2}; OPS=${4:-fill,verify,tx}; CFGS=${5:-c3_1500B,c5_imix}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for rep in $(seq 1 "$REPS"); do
  for v in main $ABS; do
    if [ "$v" = main ]; then L=$ROOT/rustnetworkstack_amd/librns_checksum.so; else L=$ROOT/tools/ab/librns_checksum_$v.so; fi
    RNS_CHECKSUM_LIB=$L timeout -k 10 300 python tools/bench_ops.py --ops "$OPS" --configs "$CFGS" \
      --out "$OUT/ops_${v}_$rep.json" > "$OUT/ops_${v}_$rep.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 "$OUT/ops_${v}_$rep.log"; exit $rc; }
    for c in ${VERIFY_CFGS:-c2_64B}; do
      RNS_CHECKSUM_LIB=$L timeout -k 10 240 python bench.py --op verify --config "$c" --steps 20 \
        > "$OUT/verify_${v}_${c}_$rep.log" 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 "$OUT/verify_${v}_${c}_$rep.log"; exit $rc; }
    done
  done
done
echo "== done"
