#!/bin/bash
# Write requests and bytes of the chain finalize (rns_tx_fill_chain_dev) and the chain fill on one
# config: rocprofv3 --pmc passes (one counter group per pass, gfx950 TCC slot limits) over
# tools/bench_ops.py with a single payload layout (one fragment).  Summarise with
#   python tools/pmc_write.py gpurun_out/<tag> --out profiles/<name>.json
# Usage: bash tools/pmc_txchain.sh <tag> <config>
set -u
TAG=${1:-pmctc}; CFG=${2:-c3_1500B}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
P=0
for ctrs in "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE"; do
  for op in tx_chain chain_fill; do
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/${op}_p$P" -o run -- \
      python3 "$ROOT/tools/bench_ops.py" --ops $op --configs $CFG --tx-frags 0 --tx-modes txpacked --steps 3 \
      --rounds 1 > "$OUT/${op}_p$P.log" 2>&1
    rc=$?; echo "$op pass $P ($ctrs) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  P=$((P+1))
done
