set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/c2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for sh in 3,4,1,2048 3,4,1,0 11,4,1,2048 11,4,1,0 11,4,1,4096 11,2,1,0 11,2,2,0 11,8,1,0 9,4,1,0; do
  timeout -k 10 120 python bench.py --config c2_64B --shape $sh --no-cpu-baseline --no-host-pipeline --steps 100 > $O/b_$sh.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "$sh rc=$rc"; exit $rc; }
  python -c "import json,sys; d=json.loads(open('$O/b_$sh.log').read().strip().splitlines()[-1]); print('$sh', d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['value'])"
done
