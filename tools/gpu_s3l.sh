#!/bin/bash
# SumVec fused XOF + eight-lane query (k_prep_w): parity, then the C3 line A/B.
set -e
O=gpurun_out/s3l
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "sumvec or wide" tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in "" "prep_fused=0" "" "prep_fused=0"; do
  opts=""; for kv in $v; do opts="$opts --opt $kv"; done
  timeout -k 10 200 python3 bench.py --role config --vdaf sumvec --no-cpu-baseline --steps 10 $opts > $O/c3.json
  python3 -c "
import json; d=json.load(open('$O/c3.json')); print('[c3 $v]', round(d['value']/1e6,3), {k: round(v['ms_avg'],3) for k,v in d.get('kernels',{}).items() if v.get('ms_avg',0)>0.02})"
done
