set -u
O=gpurun_out/r02i; mkdir -p $O
for i in 1 2; do
timeout -k 10 200 python tools/probe_lib_ab.py tools/ab/librns_checksum_old.so old >> $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
timeout -k 10 200 python tools/probe_lib_ab.py rustnetworkstack_amd/librns_checksum.so new >> $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
done
grep '^{' $O/ab.log
