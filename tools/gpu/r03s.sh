#!/bin/bash
# r03s: the jobs line at one group in flight with the launcher waiting for a quiet period
# (no job joined for Q us) before it takes an open group, Q = 0 (the r03p form) .. 800 us.
set -e
O=$PWD/gpurun_out/r03s
mkdir -p $O
run() {  # tag inflight quiet_us
  JANUS_PRIO3_MAX_INFLIGHT=$2 JANUS_PRIO3_GROUP_QUIET_US=$3 timeout -k 10 300 \
    python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_$1.json
  python3 -c "
import json; d=json.load(open('$O/jobs_$1.json')); print('[$1]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
}
for r in a b; do
  run q0_$r 1 0
  run q50_$r 1 50
  run q100_$r 1 100
  run q200_$r 1 200
  run q400_$r 1 400
  run q800_$r 1 800
done
