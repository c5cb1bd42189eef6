#!/bin/bash
# r03u: the executor's inputs prefetched to a device mirror while the previous group runs; the
# executor tests, then the jobs line (3 runs, group traces).
set -e
O=$PWD/gpurun_out/r03u
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_executor.py > $O/executor_tests.log 2>&1
tail -2 $O/executor_tests.log
for r in a b c; do
  JANUS_EXEC_TRACE=$O/trace_$r.txt timeout -k 10 300 python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_$r.json
  python3 -c "
import json; d=json.load(open('$O/jobs_$r.json')); print('[$r]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
done
