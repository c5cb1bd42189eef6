#!/bin/bash
# The 128-thread jobs line four times with the executor trace (its run-to-run spread).
set -e
OUT=${OUT:-gpurun_out/jobs128}
mkdir -p "$OUT"
for i in 1 2 3 4; do
  JANUS_EXEC_TRACE=$OUT/trace_$i.txt timeout -k 10 240 python3 bench.py --role jobs --no-cpu-baseline > "$OUT/j128_$i.json" 2> "$OUT/j128_$i.err" || { tail -20 "$OUT/j128_$i.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/j128_$i.json')); print('run $i', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
done
