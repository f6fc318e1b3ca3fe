#!/bin/bash
# One gpurun session: GPU parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit.  A test FAILURE (exit 1) does not stop the
# session; a timeout / abort / segfault (124, 134, 137, 139) does.
# Usage (from the repo root on the GPU box): bash tools/gpu_session.sh [tag] [bench args...]
set -u
TAG=${1:-r01}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"

fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }

step() {  # step <name> <timeout> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}

rocminfo 2>/dev/null | grep -m1 -E "gfx9" > "$OUT/device.txt"
nproc > "$OUT/nproc.txt"
step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py "$@"
cd /tmp
step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
     python3 "$ROOT/bench.py" --no-cpu-baseline --no-host-pipeline "$@"
# HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes, counters only (no other trace domains)
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
     python3 "$ROOT/bench.py" --no-cpu-baseline --no-host-pipeline --steps 5 --warmup 1
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
     python3 "$ROOT/bench.py" --no-cpu-baseline --no-host-pipeline --steps 5 --warmup 1
cd "$ROOT"
python tools/pmc_traffic.py --fetch "$OUT/pmc_fetch" --write "$OUT/pmc_write" --config c3_1500B \
     --kernel csum_ --algo-bytes 1574961152 --out "$OUT/traffic_c3_1500B.json" > "$OUT/traffic.log" 2>&1
echo "traffic rc=$?"; cat "$OUT/traffic.log" | tail -3
echo "== done"
