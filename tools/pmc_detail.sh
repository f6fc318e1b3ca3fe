#!/bin/bash
# L2 -> fabric read requests by size, per config: rocprofv3 PMC passes (kernel-trace only,
# each pass within the gfx950 TCC counter limit of 4).  Usage: bash tools/pmc_detail.sh <tag> [configs]
set -u
TAG=${1:-pmc}; CONFIGS=${2:-c3_1500B,c5_imix,c2_64B}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
for c in ${CONFIGS//,/ }; do
  P=1
  for ctrs in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
              "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_HIT_sum TCC_MISS_sum"; do
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/${c}_p$P" -o run -- \
      python3 "$ROOT/bench.py" --config $c --no-cpu-baseline --no-host-pipeline --steps 5 --warmup 1 > "$OUT/${c}_p$P.log" 2>&1
    rc=$?; echo "$c pass $P rc=$rc"; [ $rc -eq 0 ] || exit $rc
    P=$((P+1))
  done
done
