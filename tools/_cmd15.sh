set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r01u; mkdir -p $O; export TMPDIR=/tmp
RNS_BENCH_BACKEND=gloo RNS_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench2.log 2>&1; rc=$?; echo bench2 rc=$rc; tail -3 $O/bench2.log
