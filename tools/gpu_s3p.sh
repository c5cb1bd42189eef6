#!/bin/bash
# Prio3Count deferred slow path in one launch (k_slow_redo_gen): parity, then the C1 line A/B.
set -e
O=gpurun_out/s3p
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_executor.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in "" "slow_rpl=2" "" "slow_rpl=2" ""; do
  opts=""; for kv in $v; do opts="$opts --opt $kv"; done
  timeout -k 10 200 python3 bench.py --role config --vdaf count --no-cpu-baseline --steps 200 --warmup 20 $opts > $O/c1.json
  python3 -c "
import json; d=json.load(open('$O/c1.json')); print('[c1 $v]', round(d['value']/1e6,1), round(d['ms_per_step'],4), {k: (round(v['ms_avg'],4), v['launches']) for k,v in d.get('kernels',{}).items()})"
done
