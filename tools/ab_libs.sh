#!/bin/bash
# GPU A/B across library variants: bash tools/ab_libs.sh base ku4 occ5 ...
# ("base" = janus_amd/libjanus_prio3.so).  Prints per-kernel ms for each, same box.
for v in "$@"; do
  if [ "$v" = base ]; then unset JANUS_PRIO3_LIB; else export JANUS_PRIO3_LIB=$PWD/janus_amd/variants/libjanus_prio3_$v.so; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --warmup 5 --steps ${STEPS:-40} > gpurun_out/ab_$v.json || { echo "$v failed"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab_$v.json')); print('[$v]', round(d['value']/1e6,2), {k: round(v['ms_avg'],3) for k,v in d['kernels'].items() if v['ms_avg']>0.05}, d['checks']['finished'])"
done
