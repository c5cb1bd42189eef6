#!/bin/bash
# Prio3Sum fused XOF + query (k_prep_sum): Sum parity, then the C4 line A/B.
set -e
O=gpurun_out/s3k
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "sum" tests/test_gpu_fullsize.py tests/test_gpu_leader.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in "" "prep_fused=0" "" "prep_fused=0"; do
  opts=""; for kv in $v; do opts="$opts --opt $kv"; done
  timeout -k 10 200 python3 bench.py --role config --vdaf sum32 --no-cpu-baseline --steps 20 $opts > $O/c4.json
  python3 -c "
import json; d=json.load(open('$O/c4.json')); print('[c4 $v]', round(d['value']/1e6,2), {k: round(v['ms_avg'],3) for k,v in d.get('kernels',{}).items() if v.get('ms_avg',0)>0.02})"
done
