# Flat-kernel evaluation: parity tests, then bench.py per config for the default shape and flat shapes.
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/flat; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in c2_64B c3_1500B c5_imix c4_9000B; do
  for sh in auto 18,0,2,0 18,0,4,0 18,0,8,0; do
    if [ $sh = auto ]; then A=""; else A="--shape $sh"; fi
    timeout -k 10 120 python bench.py --config $cfg $A --no-cpu-baseline --no-host-pipeline --steps 30 > $O/b_${cfg}_$sh.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "$cfg $sh rc=$rc"; tail -3 $O/b_${cfg}_$sh.log; exit $rc; }
    python -c "import json; d=json.loads([l for l in open('$O/b_${cfg}_$sh.log') if l.startswith('{')][-1]); print('$cfg', '$sh', d['roofline']['kernel_avg_us'], d['roofline']['frac'])"
  done
done
