#!/bin/bash
# r03y: kernel + copy traces of the jobs line, the pull from the mapped staging against (A/B
# only, wrong shares) the same pull from HBM.
set -e
O=$PWD/gpurun_out/r03y
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/host -o run -- python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_host.json
JANUS_AB_PULL_FROM_DEVICE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/dev -o run -- python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_dev.json
python3 - <<'PY'
import csv, glob, statistics as st
for tag in ['host', 'dev']:
    f = glob.glob(f'gpurun_out/r03y/{tag}/**/run_kernel_stats.csv', recursive=True)
    for row in csv.DictReader(open(f[0])):
        if float(row['Percentage']) > 1:
            print(tag, row['Name'][:40], row['Calls'], round(float(row['AverageNs'])/1e3, 1), 'us avg')
PY
