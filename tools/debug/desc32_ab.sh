#!/bin/bash
# A/B of 64-bit vs compact 32-bit descriptor offsets: full GPU suite first, then
# bench.py per config, interleaved, twice.  Stops at the first failure.
set -u
TAG=${1:-d32}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; export TMPDIR=/tmp; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CFGS:-c3_1500B c5_imix c2_64B c4_9000B}; do
    for mode in u64 u32; do
      extra="--desc 64"; [ $mode = u32 ] && extra="--desc 32"
      timeout -k 10 240 python bench.py --config $cfg --no-cpu-baseline --no-host-pipeline $extra > "$OUT/bench_${cfg}_${mode}_$rep.json" 2> "$OUT/bench_${cfg}_${mode}_$rep.err"
      rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg $mode rc=$rc"; tail -5 "$OUT/bench_${cfg}_${mode}_$rep.err"; exit $rc; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['roofline']['kernel_avg_us'], d['roofline']['frac'])" "$OUT/bench_${cfg}_${mode}_$rep.json" $cfg $mode
    done
  done
done
echo "== done"
