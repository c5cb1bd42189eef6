#!/bin/bash
# k_code folded into k_acc_seg (+ 2048-report chunks for short outputs): every GPU test, then
# the C1 / C4 / C3 lines.
set -e
O=gpurun_out/s3q
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_edges.py tests/test_gpu_executor.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in count sum32 sum32; do
  st=200; [ $c = sumvec ] && st=10; [ $c = sum32 ] && st=20
  timeout -k 10 200 python3 bench.py --role config --vdaf $c --no-cpu-baseline --steps $st --warmup 5 > $O/$c.json
  python3 -c "
import json; d=json.load(open('$O/$c.json')); print('[$c]', round(d['value']/1e6,2), round(d['ms_per_step'],4), {k: (round(v['ms_avg'],4), v['launches']) for k,v in d.get('kernels',{}).items()})"
done
