set -u
O=gpurun_out/r02r; mkdir -p $O
run() { # label lib args...
  local L=$1 LIBV=$2; shift 2
  RNS_CHECKSUM_LIB=$LIBV timeout -k 10 200 python bench.py "$@" --no-cpu-baseline --no-host-pipeline > $O/b.log 2>&1 || { tail -3 $O/b.log; exit 1; }
  python -c "import json;l=[json.loads(x) for x in open('$O/b.log') if x.startswith('{')][-1];r=l['roofline'];print('$L', '$*', l['steps'], r['kernel_avg_us'], (r.get('isolated') or {}).get('kernel_avg_us'), r['frac'])" | tee -a $O/summary.txt
}
for rep in 1 2; do
  run product "" --config c3_1500B --steps 40
  run c3u3 tools/ab/librns_checksum_c3u3.so --config c3_1500B --steps 40
  run product3s "" --config c3_1500B --steps 40 --graph-streams 3
  run product "" --config c5_imix --steps 40
  run c3u3 tools/ab/librns_checksum_c3u3.so --config c5_imix --steps 40
  run product3s "" --config c5_imix --steps 40 --graph-streams 3
done
run product "" --config c2_64B --steps 200
run product3s "" --config c2_64B --steps 200 --graph-streams 3
