#!/bin/bash
# r03ag: kernel + memory-copy trace of the jobs line on the final executor (issue-ahead, output
# copy kernel), CSV summaries for profiles/.
set -e
O=$PWD/gpurun_out/r03ag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_traced.json
python3 -c "
import json; d=json.load(open('$O/jobs_traced.json')); print('[jobs traced]', round(d['value']/1e6,2), 'M/s', d['checks']['every_job_matches_cpu'])"
