set -u
O=gpurun_out/line1; mkdir -p $O
RNS_CHECKSUM_LIB=$PWD/tools/ab/librns_checksum_line.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_line.log 2>&1; rc=$?; echo "pytest line rc=$rc"; tail -3 $O/pytest_line.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh line1 "" "base line base line" csum c3_1500B,c5_imix
