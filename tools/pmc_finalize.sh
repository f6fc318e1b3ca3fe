#!/bin/bash
# HBM traffic of bench.py --op finalize as the bench runs it (batches rotating over cold header
# regions): rocprofv3 --pmc passes, one counter group per pass (gfx950 TCC slot limits).
# Summarise with: python tools/pmc_write.py gpurun_out/<tag> --out profiles/<name>.json
# Usage: bash tools/pmc_finalize.sh <tag> <config>
set -u
TAG=${1:-pmcfin}; CFG=${2:-c3_1500B}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
P=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE TCC_EA0_WRREQ_sum" "TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/finalize_p$P" -o run -- \
    python3 "$ROOT/bench.py" --op finalize --config $CFG --steps 4 --warmup 1 --ramp-s 0 --no-cpu-baseline \
    > "$OUT/finalize_p$P.log" 2>&1
  rc=$?; echo "finalize pass $P ($ctrs) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  P=$((P+1))
done
