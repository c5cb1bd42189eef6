#!/bin/bash
# r05 VERDICT item 5: the 16-thread jobs line, four runs with the executor trace and one under a
# kernel trace, to name what differs between its ~10 and ~15 M reports/s modes.
set -e
OUT=${OUT:-gpurun_out/jobs16}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2 3 4; do
  JANUS_EXEC_TRACE=$OUT/trace_$i.txt timeout -k 10 240 python3 bench.py --role jobs --threads 16 --no-cpu-baseline > "$OUT/j16_$i.json" 2> "$OUT/j16_$i.err" || { tail -20 "$OUT/j16_$i.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/j16_$i.json')); print('run $i', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --role jobs --threads 16 --no-cpu-baseline > "$OUT/j16_prof.json" 2> "$OUT/j16_prof.err" || { tail -20 "$OUT/j16_prof.err"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/j16_prof.json')); print('prof run', round(d['value']/1e6,2), 'M/s', d['coalescing'])"
