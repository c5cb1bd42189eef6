#!/bin/bash
# r03ah: the fused finish zeroes its accumulators in one kernel instead of three memsets
# (plus the r03af issue-ahead): the whole GPU suite, then the jobs line x3 with traces.
set -e
O=$PWD/gpurun_out/r03ah
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in a b c; do
  JANUS_EXEC_TRACE=$O/trace_$r.txt timeout -k 10 300 python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_$r.json
  python3 -c "
import json; d=json.load(open('$O/jobs_$r.json')); print('[jobs $r]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
done
