set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r01o; mkdir -p $O; export TMPDIR=/tmp
S="6,0,0,0;4,0,0,0;3,4,1,2048;3,2,2,2048;3,2,2,0;3,2,1,2048;1,2,2,0;3,4,2,2048"
timeout -k 10 600 python tools/sweep_shapes.py --configs c5_imix,c2_64B,d40B --shapes "$S" > $O/sweep_base.log 2>&1; echo base rc=$?
RNS_CHECKSUM_LIB=$PWD/tools/ab/librns_checksum_tinyg2.so timeout -k 10 600 python tools/sweep_shapes.py --configs c5_imix,d40B --shapes "6,0,0,0;4,0,0,0" > $O/sweep_g2.log 2>&1; echo g2 rc=$?
for f in base g2; do tail -1 $O/sweep_$f.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
for k,v in d.items(): print('$f',k, [(r['shape'], r['median_us'], r['GBps']) for r in v[:6]])"; done
