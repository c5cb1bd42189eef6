#!/bin/bash
# Jobs line (500-report jobs through the host-buffer ABI): the fused kernel vs the two-kernel
# chain vs the lane-pair XOF for the small coalesced launches, 128 and 512 threads.
set -e
O=gpurun_out/s3i
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_executor.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for T in 128 512; do
for v in "" "prep_fused=0" "xof_pair=1" "" "prep_fused=0" "xof_pair=1"; do
  opts=""; for kv in $v; do opts="$opts --opt $kv"; done
  timeout -k 10 200 python3 bench.py --role jobs --no-cpu-baseline --threads $T $opts > $O/jobs.json
  python3 -c "
import json; d=json.load(open('$O/jobs.json')); print('[T=$T $v]', round(d['value']/1e6,2), d.get('config',{}).get('launches', ''), {k: (round(v['ms_total'],1), v['launches']) for k,v in d.get('kernels',{}).items() if v.get('ms_total',0)>1})"
done
done
