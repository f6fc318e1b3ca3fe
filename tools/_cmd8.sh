set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r01n; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > $O/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 $O/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python tools/bench_ops.py --configs c3_1500B,c5_imix --rounds 3 --out $O/ops.json > $O/ops.log 2>&1; echo ops rc=$?; grep -v amdgpu $O/ops.log | grep -E "^c" | cut -c1-400
timeout -k 10 300 python tools/bench_pipeline.py --out $O/pipeline.json > $O/pipeline.log 2>&1; echo pipeline rc=$?; tail -2 $O/pipeline.log
