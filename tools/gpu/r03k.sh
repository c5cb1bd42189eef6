#!/bin/bash
# r03k: host-pull group launches (XOF reading the staging, leader shares copied under it) and
# wave-aligned aggregating jobs: executor / fused / leader tests, then the jobs line and a trace.
set -e
O=$PWD/gpurun_out/r03k
R=$PWD
mkdir -p $O
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_executor.py tests/test_gpu_fused.py tests/test_gpu_leader.py tests/test_abi.py tests/test_hpke.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for mode in combined combined two; do
  timeout -k 10 300 python3 bench.py --role jobs --jobs-call $mode --no-cpu-baseline > $O/jobs_$mode.json
  python3 -c "
import json; d=json.load(open('$O/jobs_$mode.json')); print('[$mode]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks'])"
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --role jobs --no-cpu-baseline > $O/jobs_traced.json
cd $R
timeout -k 10 200 python3 bench.py --role hpke --hpke-kem p256 --reports 262144 --steps 5 --no-cpu-baseline > $O/hpke_p256.json
python3 -c "
import json; d=json.load(open('$O/hpke_p256.json')); print('[p256]', round(d['value']/1e6,2), 'M/s', d['roofline']['frac'], d['checks'])"
