#!/bin/bash
# r03p: the in-XOF pull with coalesced per-wave pieces (1 KiB per load instruction).
set -e
O=$PWD/gpurun_out/r03p
R=$PWD
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_executor.py tests/test_gpu_fused.py tests/test_baseline_configs.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_$i.json
  python3 -c "
import json; d=json.load(open('$O/jobs_$i.json')); print('[jobs]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
done
timeout -k 10 200 python3 bench.py --role hpke --hpke-kem p256 --reports 262144 --steps 5 --no-cpu-baseline > $O/p256.json
python3 -c "
import json; d=json.load(open('$O/p256.json')); print('[p256]', round(d['value']/1e6,2), 'M/s', round(d['roofline']['frac'],3), d['checks'])"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --role jobs --no-cpu-baseline > $O/jobs_traced.json
