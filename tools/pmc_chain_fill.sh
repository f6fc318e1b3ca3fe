#!/bin/bash
# Write requests / bytes of the head-fragment chain fill on the transmit shape (VERDICT r4
# item 2: TCC_EA0_WRREQ per packet), next to the plain chain checksum of the same chains:
# rocprofv3 --pmc passes (one counter group per pass) over tools/bench_ops.py --ops chain_fill.
# Usage: bash tools/pmc_chain_fill.sh <tag> [configs] [modes]; then python tools/pmc_write.py gpurun_out/<tag>
set -u
TAG=${1:-pmccf}; CFGS=${2:-c3_1500B,c5_imix}; MODES=${3:-txpacked,plain}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
P=0
for ctrs in "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE"; do
  for cfg in ${CFGS//,/ }; do
    timeout -s KILL 150 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/${cfg}_p$P" -o run -- \
      python3 "$ROOT/tools/bench_ops.py" --ops chain_fill --configs $cfg --tx-frags 0 --tx-modes $MODES \
      --steps 2 --rounds 1 > "$OUT/${cfg}_p$P.log" 2>&1
    rc=$?; echo "$cfg pass $P ($ctrs) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  P=$((P+1))
done
