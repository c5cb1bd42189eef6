#!/bin/bash
# the jobs lines with the executor's group trace (JANUS_EXEC_TRACE), plain
# and under a rocprofv3 kernel + memory-copy trace, so a fast and a slow run can be told apart by
# group sizes, launch durations, queues and host staging time.
#   OUT=gpurun_out/<tag> bash tools/gpu/trace_lines.sh [ROLE [PLAIN [TRACED [THREADS]]]]
# ROLE: helper (default) | leader | init
set -e
OUT=${OUT:-gpurun_out/trace}
ROLE=${1:-helper}
PLAIN=${2:-3}
TRACED=${3:-2}
T=${4:-128}
mkdir -p "$OUT"
export TMPDIR=/tmp
summ() {
  python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['value']/1e6,3), 'M/s', d['coalescing'], {k: v for k, v in d['checks'].items() if isinstance(v, bool)}, (d.get('two_call') or {}).get('value'))"
}
for i in $(seq 1 "$PLAIN"); do
  JANUS_EXEC_TRACE=$OUT/${ROLE}_t${T}_plain_$i.trace timeout -k 10 300 python3 bench.py --role jobs --jobs-role "$ROLE" --threads "$T" --no-cpu-baseline > "$OUT/${ROLE}_t${T}_plain_$i.json" 2> "$OUT/${ROLE}_t${T}_plain_$i.err" || { tail -20 "$OUT/${ROLE}_t${T}_plain_$i.err"; exit 1; }
  summ "$OUT/${ROLE}_t${T}_plain_$i.json" "plain $i"
done
for i in $(seq 1 "$TRACED"); do
  JANUS_EXEC_TRACE=$OUT/${ROLE}_t${T}_prof_$i.trace timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/${ROLE}_t${T}_prof_$i" -o run -- python3 bench.py --role jobs --jobs-role "$ROLE" --threads "$T" --no-cpu-baseline > "$OUT/${ROLE}_t${T}_prof_$i.json" 2> "$OUT/${ROLE}_t${T}_prof_$i.err" || { tail -20 "$OUT/${ROLE}_t${T}_prof_$i.err"; exit 1; }
  summ "$OUT/${ROLE}_t${T}_prof_$i.json" "traced $i"
done
