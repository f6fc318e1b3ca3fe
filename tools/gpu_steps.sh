#!/bin/bash
# Run named GPU steps, each under its own time limit, logs under gpurun_out/<tag>/.
# A fatal status (timeout 124/137, abort 134, segfault 139) stops the session; an
# ordinary failure is reported and the session goes on.
#   bash tools/gpu_steps.sh <tag> <name> <timeout_s> "<command>" [<name> <timeout_s> "<command>" ...]
# Commands run from the repo root with TMPDIR=/tmp; a command starting with "prof:" runs
# `rocprofv3 --kernel-trace --stats` around the rest (from /tmp, output in <tag>/<name>_prof)
# and reconciles it with tools/profile_bench.py.  "@ROOT@" in a command = the repo root.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
while [ $# -ge 3 ]; do
  name=$1; lim=$2; cmd=${3//@ROOT@/$ROOT}; shift 3
  echo "== $name ($(date +%T))"
  if [ "${cmd#prof:}" != "$cmd" ]; then
    cmd=${cmd#prof:}
    (cd /tmp && timeout -k 10 "$lim" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${name}_prof" -o run -- \
        $cmd > "$OUT/$name.log" 2>&1)
    rc=$?
    if [ $rc -eq 0 ]; then
      python tools/profile_bench.py --trace "$OUT/${name}_prof/run_kernel_trace.csv" \
        --stats "$OUT/${name}_prof/run_kernel_stats.csv" --bench "$OUT/$name.log" \
        --out "$OUT/rocprof_$name.json" --timed-stats-out "$OUT/rocprof_${name}_timed_stats.csv" > "$OUT/${name}_pb.log" 2>&1
      echo "   profile_bench rc=$?"
    fi
  else
    timeout -k 10 "$lim" bash -c "$cmd" > "$OUT/$name.log" 2>&1
    rc=$?
  fi
  echo "   rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-600
  case $rc in 124|134|137|139) echo "FATAL rc=$rc in $name: stopping"; exit $rc;; esac
done
echo "== done"
