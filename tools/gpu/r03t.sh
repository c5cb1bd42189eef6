#!/bin/bash
# r03t: executor group traces (JANUS_EXEC_TRACE) of the jobs line at Q = 0 and 100 us.
set -e
O=$PWD/gpurun_out/r03t
mkdir -p $O
for q in 0 100; do
  JANUS_EXEC_TRACE=$O/trace_q$q.txt JANUS_PRIO3_GROUP_QUIET_US=$q timeout -k 10 300 \
    python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_q$q.json
  python3 -c "
import json; d=json.load(open('$O/jobs_q$q.json')); print('[q$q]', round(d['value']/1e6,2), 'M/s', d['coalescing'])"
done
