set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r01t; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_fill.py tests/test_gpu_rx.py -x -q -m gpu > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in main g64 g128; do
  if [ $v = main ]; then L=$PWD/rustnetworkstack_amd/librns_checksum.so; else L=$PWD/tools/ab/librns_checksum_$v.so; fi
  RNS_CHECKSUM_LIB=$L timeout -k 10 300 python -m pytest tests/test_gpu_fill.py -x -q -m gpu > $O/pytest_$v.log 2>&1; rc=$?; echo $v fill-tests rc=$rc
  [ $rc -eq 0 ] || exit $rc
  RNS_CHECKSUM_LIB=$L timeout -k 10 300 python tools/bench_ops.py --ops fill --configs c3_1500B,c5_imix,c4_9000B > $O/ops_$v.log 2>&1; rc=$?; echo $v ops rc=$rc; tail -1 $O/ops_$v.log
  [ $rc -eq 0 ] || exit $rc
done
