#!/bin/bash
# r03r: the jobs line with the quiet-period lookahead launcher (2 groups in flight) against one
# group in flight, interleaved; then the executor tests.
set -e
O=$PWD/gpurun_out/r03r
mkdir -p $O
run() {  # tag inflight quiet_us
  JANUS_PRIO3_MAX_INFLIGHT=$2 JANUS_PRIO3_GROUP_QUIET_US=$3 timeout -k 10 300 \
    python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_$1.json
  python3 -c "
import json; d=json.load(open('$O/jobs_$1.json')); print('[$1]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
}
for r in a b; do
  run inf1_$r 1 100
  run inf2_q50_$r 2 50
  run inf2_q100_$r 2 100
  run inf2_q200_$r 2 200
  run inf2_q400_$r 2 400
done
JANUS_PRIO3_MAX_INFLIGHT=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_executor.py > $O/executor_tests.log 2>&1
tail -2 $O/executor_tests.log
