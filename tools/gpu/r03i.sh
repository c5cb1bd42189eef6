#!/bin/bash
# r03i: host->device bandwidth (pinned copies vs a kernel reading mapped host memory), and the
# fused prepare kernel's time against batch size (the jobs line runs 20-30k-report groups).
set -e
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 120 ./tools/ubench_h2d | tee $O/h2d.txt
for n in 16384 32768 65536 131072 196608 262144; do
  timeout -k 10 120 python3 bench.py --reports $n --steps 20 --warmup 3 --no-cpu-baseline > $O/c2_$n.json
  python3 -c "
import json; d=json.load(open('$O/c2_$n.json')); print($n, round(d['value']/1e6,2), 'M/s', {k: round(v['ms_avg'],3) for k,v in d['kernels'].items()})"
done
