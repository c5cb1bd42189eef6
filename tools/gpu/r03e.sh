#!/bin/bash
# r03e: the combined prepare+aggregate host call -- executor tests, then the jobs line with one
# and with two round trips per job (every job checked against the oracle).
set -e
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_executor.py tests/test_abi.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for mode in combined two; do
  timeout -k 10 300 python3 bench.py --role jobs --jobs-call $mode --no-cpu-baseline > $O/jobs_$mode.json
  python3 -c "
import json; d=json.load(open('$O/jobs_$mode.json')); print('[$mode]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks'])"
done
