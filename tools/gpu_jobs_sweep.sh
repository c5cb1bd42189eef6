#!/bin/bash
# bench.py --role jobs over host threads x executor in-flight groups (x job size)
mkdir -p gpurun_out
T=${1:-r02f}
for js in ${JOB_SIZES:-500}; do for th in ${THREADS:-16 64 128}; do for inf in ${INFLIGHT:-1 2 4}; do
  JANUS_PRIO3_MAX_INFLIGHT=$inf timeout -k 10 200 python -u bench.py --role jobs --no-cpu-baseline --threads $th --job-size $js \
    > gpurun_out/${T}_jobs_j${js}_t${th}_i${inf}.json 2> gpurun_out/${T}_jobs.err || { echo "jobs failed"; tail -20 gpurun_out/${T}_jobs.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_jobs_j${js}_t${th}_i${inf}.json')); print('job', $js, 'threads', $th, 'inflight', $inf, round(d['value']/1e6,2), 'M/s', 'rep/launch', round(d['coalescing']['mean_reports_per_launch']), d['checks'])"
done; done; done
