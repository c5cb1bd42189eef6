#!/bin/bash
# Interleaved A/B of bench lines over values of one environment variable (the in-tree library):
#   OUT=... bash tools/gpu/ab_env.sh VAR "VALUES" REPS NAME:ARGS [NAME:ARGS ...]
# (ARGS ','-separated; the value '-' leaves VAR unset; TRACE=1: each run's JANUS_EXEC_TRACE beside it)
set -e
OUT=${OUT:-gpurun_out/ab_env}
mkdir -p "$OUT"
VAR=$1; VALS=$2; REPS=$3; shift 3
for rep in $(seq $REPS); do
  for line in "$@"; do
    name=${line%%:*}; args=${line#*:}
    for v in $VALS; do
      if [ "$v" = - ]; then unset $VAR; else export $VAR=$v; fi
      if [ -n "$TRACE" ]; then export JANUS_EXEC_TRACE=$OUT/${name}_${v}_$rep.trace; fi
      timeout -k 10 240 python3 bench.py ${args//,/ } > "$OUT/${name}_${v}_$rep.json" 2> "$OUT/${name}_${v}_$rep.err" || { tail -20 "$OUT/${name}_${v}_$rep.err"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/${name}_${v}_$rep.json')); print('$name $VAR=$v $rep', round(d['value']/1e6,2), d.get('coalescing'))"
    done
  done
done
unset $VAR
