#!/bin/bash
# r03q: the jobs line with 1, 2 and 3 groups in flight (the XOF pulls its own inputs now).
set -e
O=$PWD/gpurun_out/r03q
mkdir -p $O
for inf in 1 2 3 1 2 3; do
  JANUS_PRIO3_MAX_INFLIGHT=$inf timeout -k 10 300 python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_inf$inf.json
  python3 -c "
import json; d=json.load(open('$O/jobs_inf$inf.json')); print('[inflight $inf]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
done
