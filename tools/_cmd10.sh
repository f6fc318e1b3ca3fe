set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r01p; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_rx.py tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q -m gpu > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_ops.py --out $O/ops.json > $O/ops.log 2>&1; rc=$?; echo ops rc=$rc; tail -3 $O/ops.log
