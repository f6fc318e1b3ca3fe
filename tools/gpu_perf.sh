#!/bin/bash
# One gpurun session of measurements: bench.py on every BASELINE.json GPU config and
# tools/bench_ops.py (chain / fill / verify beside the plain batch).  Each GPU step has
# its own time limit; a timeout / abort / segfault stops the session.
# Usage (repo root on the GPU box): bash tools/gpu_perf.sh <tag> [configs] [ops-configs]
set -u
TAG=${1:-perf}
CONFIGS=${2:-c2_64B,c3_1500B,c4_9000B,c5_imix}
OPSCFG=${3:-c3_1500B,c5_imix}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"

step() {  # step <name> <timeout> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 2 "$OUT/$name.log"
  case $rc in 0|1) ;; *) echo "FATAL rc=$rc in $name: stopping"; exit $rc;; esac
}

for c in ${CONFIGS//,/ }; do
  step "bench_$c" 300 python bench.py --config "$c" --cpu-seconds 5 --no-host-pipeline
done
if [ -n "$OPSCFG" ]; then
  step ops 400 python tools/bench_ops.py --configs "$OPSCFG" --out "$OUT/ops.json"
fi
echo "== done"
