#!/bin/bash
# Redo launches scanning 64 flags per lane: slow-path parity, then C2 / C1 tails.
set -e
O=gpurun_out/s3v
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_edges.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 40 --warmup 5 > $O/c2.json
python3 -c "
import json; d=json.load(open('$O/c2.json')); print('[c2]', round(d['value']/1e6,2), round(d['ms_per_step'],4), {k: round(v['ms_avg'],4) for k,v in d.get('kernels',{}).items()})"
for v in count sum32; do
timeout -k 10 200 python3 bench.py --role config --vdaf $v --no-cpu-baseline --steps 100 --warmup 10 > $O/$v.json
python3 -c "
import json; d=json.load(open('$O/$v.json')); print('[$v]', round(d['value']/1e6,2), round(d['ms_per_step'],4), {k: round(v['ms_avg'],4) for k,v in d.get('kernels',{}).items()})"
done
