#!/bin/bash
# k_agg_waves with one wave-segment load per lane and unconditional chunk loads: fused-accumulate
# parity, then the C2 line's tail kernels.
set -e
O=gpurun_out/s3u
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_executor.py tests/test_batch_metadata.py tests/test_gpu_leader.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 40 --warmup 5 > $O/c2.json
  python3 -c "
import json; d=json.load(open('$O/c2.json')); print('[c2]', round(d['value']/1e6,2), round(d['ms_per_step'],4), {k: round(v['ms_avg'],4) for k,v in d.get('kernels',{}).items()})"
done
