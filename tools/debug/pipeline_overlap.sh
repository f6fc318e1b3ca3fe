#!/bin/bash
# Batched receive / transmit pipelines, synchronous vs overlapped (two buffer sets), 3 reps each.
set -u
O=gpurun_out/${1:-pipe3}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
for mode in "" "--overlap" "--tx" "--tx --overlap"; do
  tag=$(echo "rx $mode" | tr -d '-' | tr ' ' '_')_$rep
  timeout -k 10 200 python tools/bench_pipeline.py --packets 1048576 $mode --out $O/$tag.json > $O/$tag.log 2>&1; rc=$?; echo "$mode rc=$rc"; tail -1 $O/$tag.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
done
