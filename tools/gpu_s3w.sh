#!/bin/bash
# Final state: whole GPU suite, smoke(), the headline line with its CPU baseline, rocprof stats.
set -e
O=gpurun_out/s3w
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/c2.json
python3 -c "
import json; d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]); print('[c2]', round(d['value']/1e6,2), round(d['ms_per_step'],4), d['roofline'].get('frac'), (d.get('cpu_baseline') or {}).get('value'), d.get('checks'))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -12 $O/kernel_stats.csv
