set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r01b; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/r01b/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -5 gpurun_out/r01b/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python tools/sweep_shapes.py > gpurun_out/r01b/sweep.log 2>&1; rc=$?; echo sweep rc=$rc; grep -v amdgpu.ids gpurun_out/r01b/sweep.log | head -5
