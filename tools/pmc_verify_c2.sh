#!/bin/bash
# PMC attribution of 64-byte receive verify: the strided receive kernel
# (bench.py --op verify, c2) and the packed entry's stream-kernel ACK path (--desc packed) against
# the strided tiny checksum of the same bytes (bench.py c2): SQ issue / wait / busy cycles, VALU,
# VMEM and LDS instructions.  One --pmc pass per counter group (gfx950 block limits), kernel
# counters only.  Usage (GPU box, repo root): bash tools/pmc_verify_c2.sh <tag>;
# summary: python tools/pmc_verify_c2.py gpurun_out/<tag>
set -u
TAG=${1:-pmcv2}; ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
P=1
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
            "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES"; do
  for who in csum verify verify_packed; do
    case $who in
      csum) args="--config c2_64B";;
      verify) args="--op verify --config c2_64B";;
      verify_packed) args="--op verify --config c2_64B --desc packed";;
    esac
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/${who}_p$P" -o run -- \
      python3 "$ROOT/bench.py" $args --no-cpu-baseline --no-host-pipeline --ramp-s 0 --steps 5 --warmup 1 \
      > "$OUT/${who}_p$P.log" 2>&1
    rc=$?; echo "$who pass $P rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  P=$((P+1))
done
echo "== done"
