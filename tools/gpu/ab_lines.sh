#!/bin/bash
# Interleaved A/B of bench lines between the in-tree library and variants:
#   OUT=... bash tools/gpu/ab_lines.sh "VARIANTS" REPS NAME:ARGS [NAME:ARGS ...]
# (ARGS ','-separated; 'base' = the in-tree library)
set -e
OUT=${OUT:-gpurun_out/ab_lines}
mkdir -p "$OUT"
VARS=$1; REPS=$2; shift 2
for rep in $(seq $REPS); do
  for line in "$@"; do
    name=${line%%:*}; args=${line#*:}
    for v in $VARS; do
      if [ "$v" = base ]; then unset JANUS_PRIO3_LIB; else export JANUS_PRIO3_LIB=$PWD/janus_amd/variants/libjanus_prio3_$v.so; fi
      timeout -k 10 240 python3 bench.py ${args//,/ } > "$OUT/${name}_${v}_$rep.json" 2> "$OUT/${name}_${v}_$rep.err" || { tail -20 "$OUT/${name}_${v}_$rep.err"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/${name}_${v}_$rep.json')); print('$name $v $rep', round(d['value']/1e6,2), d.get('coalescing'))"
    done
  done
done
