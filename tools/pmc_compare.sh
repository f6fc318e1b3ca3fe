#!/bin/bash
# PMC comparison of the streaming read probe (tools/store_probe, "read" = read_store<0,2>)
# with the headline c3 kernel: SQ issue/wait cycles, TA/TCP stalls, L1->L2 read requests.
# One --pmc pass per counter group (gfx950 block limits), kernel-trace only.
# Usage (GPU box, repo root): bash tools/pmc_compare.sh <tag>; summary: python tools/pmc_compare.py gpurun_out/<tag>
set -u
TAG=${1:-pmccmp}; ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
P=1
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
            "SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM" \
            "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"; do
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/probe_p$P" -o run -- "$ROOT/tools/store_probe" \
    > "$OUT/probe_p$P.log" 2>&1
  rc=$?; echo "probe pass $P rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/c3_p$P" -o run -- \
    python3 "$ROOT/bench.py" --config c3_1500B --no-cpu-baseline --no-host-pipeline --steps 5 --warmup 1 > "$OUT/c3_p$P.log" 2>&1
  rc=$?; echo "c3 pass $P rc=$rc"; [ $rc -eq 0 ] || exit $rc
  P=$((P+1))
done
echo "== done"
