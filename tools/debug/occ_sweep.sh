set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/occ; export TMPDIR=/tmp
timeout -k 10 300 python tools/sweep_shapes.py --configs c3_1500B --shapes "6,0,0,0;262,0,0,0;518,0,0,0;774,0,0,0;1030,0,0,0;1286,0,0,0;3,32,4,0;259,32,4,0;515,32,4,0;771,32,4,0;1027,32,4,0" --rounds 3 --iters 10 > gpurun_out/occ/c3.log 2>&1 || exit $?
timeout -k 10 300 python tools/sweep_shapes.py --configs c5_imix --shapes "4,0,0,0;260,0,0,0;516,0,0,0;772,0,0,0" --rounds 3 --iters 10 > gpurun_out/occ/c5.log 2>&1 || exit $?
timeout -k 10 300 python tools/sweep_shapes.py --configs c4_9000B --shapes "2,64,4,0;258,64,4,0;514,64,4,0;1026,64,4,0;1538,64,4,0" --rounds 3 --iters 10 > gpurun_out/occ/c4.log 2>&1 || exit $?
