set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r01i; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_session.sh r01i --steps 50 --warmup 5 --cpu-seconds 10 || exit $?
for c in c2_64B c4_9000B c5_imix; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --no-host-pipeline --cpu-seconds 3 > $O/bench_$c.log 2>&1; rc=$?; echo bench $c rc=$rc
  case $rc in 124|134|137|139) exit $rc;; esac
done
timeout -k 10 600 python tools/sweep_shapes.py --configs c5_imix,d40B,c2_64B --shapes "6,0,0,0;4,0,0,0;3,4,1,2048;1,8,2,0;3,4,1,0;1,4,1,0" > $O/sweep.log 2>&1; echo sweep rc=$?
