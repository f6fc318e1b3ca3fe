set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r01r; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_rx.py tests/test_gpu_parity.py tests/test_gpu_fill.py -x -q -m gpu > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in main occ3 nopf nopf_occ3; do
  if [ $v = main ]; then L=$PWD/rustnetworkstack_amd/librns_checksum.so; else L=$PWD/tools/ab/librns_checksum_$v.so; fi
  RNS_CHECKSUM_LIB=$L timeout -k 10 300 python tools/sweep_shapes.py --configs c5_imix,c3_1500B,c2_64B --shapes "4,0,0,0;6,0,0,0" > $O/sweep_$v.log 2>&1; rc=$?; echo $v sweep rc=$rc
  [ $rc -eq 0 ] || exit $rc
  tail -1 $O/sweep_$v.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
for k,v in d.items(): print('$v',k, [(r['shape'], r['median_us']) for r in v[:6]])"
  RNS_CHECKSUM_LIB=$L timeout -k 10 300 python tools/bench_ops.py --ops verify,fill > $O/ops_$v.log 2>&1; rc=$?; echo $v ops rc=$rc; tail -1 $O/ops_$v.log
  [ $rc -eq 0 ] || exit $rc
done
