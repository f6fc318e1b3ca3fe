#!/bin/bash
# bench.py A/B of library builds: the driver's timed region (graph replay, rotating
# batches) for each build, alternating, REPS times; one summary line per run.
# Usage: bash tools/bench_ab.sh <tag> <config> <steps> "<ab names>" [reps]
set -u
TAG=$1; CFG=$2; K=$3; ABS=$4; REPS=${5:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for rep in $(seq 1 "$REPS"); do
  for v in main $ABS; do
    if [ "$v" = main ]; then L=$ROOT/rustnetworkstack_amd/librns_checksum.so; else L=$ROOT/tools/ab/librns_checksum_$v.so; fi
    RNS_CHECKSUM_LIB=$L timeout -k 10 240 python bench.py --config "$CFG" --steps "$K" --no-cpu-baseline --no-host-pipeline \
      > "$OUT/b_${v}_$rep.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 "$OUT/b_${v}_$rep.log"; exit $rc; }
    python -c "import json;l=[json.loads(x) for x in open('$OUT/b_${v}_$rep.log') if x.startswith('{')][-1];r=l['roofline'];print('$v', '$CFG', l['ms_per_step'], r['kernel_avg_us'], (r.get('isolated') or {}).get('kernel_avg_us'), r['frac'], l['cpu_baseline'] if False else '')" | tee -a "$OUT/summary.txt"
  done
done
echo "== done"
