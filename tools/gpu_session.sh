#!/bin/bash
# One gpurun session: GPU parity tests, smoke, the driver's bench command, and a
# rocprofv3 kernel trace of THAT SAME command (reconciled by tools/profile_bench.py),
# then PMC traffic passes.  Each GPU step has its own time limit.  A test FAILURE
# (exit 1) does not stop the session; a timeout / abort / segfault (124, 134, 137,
# 139) does.
# Usage (from the repo root on the GPU box): bash tools/gpu_session.sh [tag] [config] [steps] [warmup]
set -u
TAG=${1:-r02}
CONFIG=${2:-c3_1500B}
STEPS=${3:-20}
WARMUP=${4:-5}
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
cat /sys/fs/cgroup/cpu.max > "$OUT/cpu_max.txt" 2>/dev/null
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
# the driver's command, profiled: the bench line and the kernel trace come from ONE run
cd /tmp
step bench_prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
     python3 "$ROOT/bench.py" --gpus 1 --steps "$STEPS" --warmup "$WARMUP" --config "$CONFIG"
cd "$ROOT"
python tools/profile_bench.py --trace "$OUT/prof/run_kernel_trace.csv" --stats "$OUT/prof/run_kernel_stats.csv" \
     --bench "$OUT/bench_prof.log" --out "$OUT/rocprof_bench_$CONFIG.json" --timed-stats-out "$OUT/rocprof_bench_${CONFIG}_timed_stats.csv" > "$OUT/profile_bench.log" 2>&1
echo "profile_bench rc=$?"; tail -2 "$OUT/profile_bench.log"
if [ -z "${SKIP_PMC:-}" ]; then
  cd /tmp
  # HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes, counters only (no other trace domains)
  step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
       python3 "$ROOT/bench.py" --no-cpu-baseline --no-host-pipeline --ramp-s 0 --steps 5 --warmup 1 --config "$CONFIG"
  step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
       python3 "$ROOT/bench.py" --no-cpu-baseline --no-host-pipeline --ramp-s 0 --steps 5 --warmup 1 --config "$CONFIG"
  cd "$ROOT"
  ALGO=$(python -c "import json;print([json.loads(l) for l in open('$OUT/bench_prof.log') if l.startswith('{')][-1]['roofline']['algorithmic_bytes_per_launch'])")
  python tools/pmc_traffic.py --fetch "$OUT/pmc_fetch" --write "$OUT/pmc_write" --config "$CONFIG" \
       --kernel csum_ --algo-bytes "$ALGO" --out "$OUT/traffic_$CONFIG.json" > "$OUT/traffic.log" 2>&1
  echo "traffic rc=$?"; tail -3 "$OUT/traffic.log"
fi
echo "== done"
