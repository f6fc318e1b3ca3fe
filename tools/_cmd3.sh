set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r01j; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -5 $O/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 120 ./tools/hbm_read_probe > $O/probe.log 2>&1; rc=$?; echo probe rc=$rc
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python tools/sweep_shapes.py --configs c5_imix,c3_1500B,d576B,c2_64B --shapes "6,0,0,0;4,0,0,0;3,32,4,0;3,16,4,0;1,8,2,0;3,4,1,2048" > $O/sweep.log 2>&1; rc=$?; echo sweep rc=$rc; grep -v amdgpu.ids $O/sweep.log | head -4 | cut -c1-600
