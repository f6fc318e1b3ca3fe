set -u
mkdir -p gpurun_out/r02c
timeout -k 10 300 python -u -m pytest tests/test_gpu_chains.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02c/chains.log 2>&1 || { tail -30 gpurun_out/r02c/chains.log; exit 1; }
tail -3 gpurun_out/r02c/chains.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02c/gpu.log 2>&1 || { tail -30 gpurun_out/r02c/gpu.log; exit 1; }
tail -2 gpurun_out/r02c/gpu.log
timeout -k 10 300 python tools/bench_ops.py --ops csum,chain --out gpurun_out/r02c/ops_chain.json > gpurun_out/r02c/ops.log 2>&1; echo ops rc=$?
tail -20 gpurun_out/r02c/ops.log
