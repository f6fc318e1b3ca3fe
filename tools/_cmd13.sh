set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r01s; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_ops.py --ops csum,verify > $O/ops.log 2>&1; rc=$?; echo ops rc=$rc; tail -1 $O/ops.log
