#!/bin/bash
# Issue / wait / instruction-fetch counters of the bench kernel for given configs:
# SQ wave-cycle split, instruction counts and the SQC instruction cache.  One --pmc
# pass per counter group, kernel-trace only, each under its own time limit.
# Usage (GPU box, repo root): [BENCH_EXTRA="--op verify"] bash tools/pmc_issue.sh <tag> [configs...];
# summary: python tools/pmc_issue.py gpurun_out/<tag>
set -u
TAG=${1:-pmciss}; shift; CONFIGS=${@:-c5_imix c3_1500B}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
for c in $CONFIGS; do
  P=1
  for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_IFETCH" \
              "SQC_ICACHE_REQ SQC_ICACHE_MISSES" "SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE" \
              "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH_LEVEL SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES"; do
    timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/${c}_p$P" -o run -- \
      python3 "$ROOT/bench.py" --config "$c" --no-cpu-baseline --no-host-pipeline --ramp-s 0 --steps 5 --warmup 1 ${BENCH_EXTRA:-} \
      > "$OUT/${c}_p$P.log" 2>&1
    rc=$?; echo "$c pass $P rc=$rc"; [ $rc -eq 0 ] || exit $rc
    P=$((P+1))
  done
done
echo "== done"
