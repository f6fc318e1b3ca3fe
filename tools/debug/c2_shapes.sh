# 64 B batches (cache-cold rotation in bench.py): rounds kernel shapes and grid caps.
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/c2b; mkdir -p $O; export TMPDIR=/tmp
for sh in 3,4,1,2048 3,4,1,1024 3,4,1,4096 3,4,1,512 11,4,1,1024 11,4,1,2048 11,4,1,512 3,4,2,1024 11,4,2,1024 3,8,1,2048 6,0,0,2048; do
  timeout -k 10 120 python bench.py --config c2_64B --shape $sh --no-cpu-baseline --no-host-pipeline --steps 100 > $O/b_$sh.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "$sh rc=$rc"; exit $rc; }
  python -c "import json; d=json.loads([l for l in open('$O/b_$sh.log') if l.startswith('{')][-1]); print('$sh', d['roofline']['kernel_avg_us'], d['roofline']['frac'])"
done
