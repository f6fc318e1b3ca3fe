set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r01q; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_rx.py tests/test_gpu_pipeline.py -x -q -m gpu > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_ops.py --ops verify,csum > $O/ops_nt.log 2>&1; rc=$?; echo nt rc=$rc; tail -1 $O/ops_nt.log
[ $rc -eq 0 ] || exit $rc
RNS_CHECKSUM_LIB=$PWD/tools/ab/librns_checksum_rxplain.so timeout -k 10 300 python tools/bench_ops.py --ops verify > $O/ops_plain.log 2>&1; rc=$?; echo plain rc=$rc; tail -1 $O/ops_plain.log
