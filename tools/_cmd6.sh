set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r01l; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python tools/bench_ops.py --out $O/ops.json > $O/ops.log 2>&1; rc=$?; echo ops rc=$rc; grep -v amdgpu $O/ops.log | tail -3
