#!/bin/bash
# HBM traffic (PMC FETCH_SIZE / WRITE_SIZE, one counter per pass, no trace domains) of the
# bench kernel for each config -> gpurun_out/<tag>/traffic_<config>.json, the file
# bench.py reads for roofline.traffic once copied to profiles/.
# Usage (GPU box, repo root): bash tools/pmc_configs.sh <tag> [configs]
set -u
TAG=${1:-pmc}; CONFIGS=${2:-c2_64B,c4_9000B,c5_imix}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in ${CONFIGS//,/ }; do
  cd /tmp
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/${c}_$ctr" -o run -- \
      python3 "$ROOT/bench.py" --config $c --no-cpu-baseline --no-host-pipeline --steps 5 --warmup 1 \
      > "$OUT/${c}_$ctr.log" 2>&1
    rc=$?; echo "$c $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  cd "$ROOT"
  algo=$(python3 -c "from rustnetworkstack_amd.workloads import make_layout; l = make_layout('$c'); print(int(l.payload_bytes) + 2 * l.n)")
  python3 tools/pmc_traffic.py --fetch "$OUT/${c}_FETCH_SIZE" --write "$OUT/${c}_WRITE_SIZE" --config $c \
    --kernel csum_ --algo-bytes "$algo" --out "$OUT/traffic_$c.json" > "$OUT/traffic_$c.log" 2>&1
  echo "$c traffic rc=$? algo=$algo"; tail -n 2 "$OUT/traffic_$c.log"
done
echo "== done"
