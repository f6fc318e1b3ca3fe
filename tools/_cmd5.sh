set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r01k; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > $O/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -5 $O/pytest_gpu.log
