#!/bin/bash
# Round-3 end evidence (d, after the executor's issue-ahead): smoke() and the jobs line with its
# CPU baseline and every job checked against the restatement, into gpurun_out/final3d/.
set -e
O=gpurun_out/final3d
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in a b; do
  timeout -k 10 400 python3 bench.py --role jobs > $O/jobs128_$r.json
  python3 -c "
import json; d=json.load(open('$O/jobs128_$r.json')); print('[jobs $r]', round(d['value']/1e6,2), 'M/s', d['roofline']['frac'], d['cpu_baseline']['value'], d['checks']['every_job_matches_cpu'])"
done
