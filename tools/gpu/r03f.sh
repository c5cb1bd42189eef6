#!/bin/bash
# r03f: the combined host-buffer jobs line vs launches in flight (1/2/3), then its kernel +
# copy trace.
set -e
O=$PWD/gpurun_out/r03f
mkdir -p $O
for inf in 1 2 3; do
  JANUS_PRIO3_MAX_INFLIGHT=$inf timeout -k 10 300 python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_inf$inf.json
  python3 -c "
import json; d=json.load(open('$O/jobs_inf$inf.json')); print('[inflight $inf]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --role jobs --no-cpu-baseline > $O/jobs_traced.json
ls $O/trace/*/ | head
