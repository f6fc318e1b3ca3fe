# N>1 rehearsal on ONE GPU (2 ranks share device 0 over gloo): c3 weak, c5 strong.
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-mr}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c5_imix --no-host-pipeline --cpu-seconds 3 > $O/c5_n1.log 2>&1; rc=$?; echo c5 n1 rc=$rc; tail -1 $O/c5_n1.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
for cfg in c3_1500B c5_imix; do
  RNS_BENCH_BACKEND=gloo RNS_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --config $cfg > $O/${cfg}_n2.log 2>&1
  rc=$?; echo $cfg n2 rc=$rc; grep '^{' $O/${cfg}_n2.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
done
