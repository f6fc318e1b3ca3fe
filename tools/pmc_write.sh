#!/bin/bash
# Write (and read) traffic of the transmit fill / finalize kernels next to the plain
# checksum on c3: rocprofv3 --pmc passes, one counter group per pass
# (gfx950 TCC slot limits), over tools/bench_ops.py --ops <op>.
# Usage: bash tools/pmc_write.sh <tag> [ops] [config]; then python tools/pmc_write.py gpurun_out/<tag>
set -u
TAG=${1:-pmcw}; OPS=${2:-csum,fill,tx}; CFG=${3:-c3_1500B}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
P=0
for ctrs in "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" \
            "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"; do
  for op in ${OPS//,/ }; do
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/${op}_p$P" -o run -- \
      python3 "$ROOT/tools/bench_ops.py" --ops $op --configs $CFG --steps 3 --rounds 1 > "$OUT/${op}_p$P.log" 2>&1
    rc=$?; echo "$op pass $P ($ctrs) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  P=$((P+1))
done
