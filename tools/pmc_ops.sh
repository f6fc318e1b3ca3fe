#!/bin/bash
# HBM bytes (FETCH_SIZE, WRITE_SIZE: separate rocprofv3 --pmc passes) of any tools/bench_ops.py
# op, e.g. the chain checksum on 512-byte NetBuffers:
#   bash tools/pmc_ops.sh <tag> chain c5_imix --chain-layouts netbuf
# then python tools/pmc_write.py gpurun_out/<tag> (per-kernel sums per dispatch).
set -u
TAG=$1; OPS=$2; CFGS=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
P=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE"; do
  for cfg in ${CFGS//,/ }; do
    timeout -s KILL 150 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/${cfg}_p$P" -o run -- \
      python3 "$ROOT/tools/bench_ops.py" --ops "$OPS" --configs $cfg --steps 2 --rounds 1 "$@" > "$OUT/${cfg}_p$P.log" 2>&1
    rc=$?; echo "$cfg pass $P ($ctrs) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  P=$((P+1))
done
