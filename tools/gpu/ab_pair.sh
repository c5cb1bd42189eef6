#!/bin/bash
# r05 A/B of the lane-pair prepare (k_prep_hp) at the full-chip 1 Mi batch against the one-lane
# k_prep_h: parity of every variant on the Histogram tests, then interleaved bench steps.
#   OUT=gpurun_out/<tag> bash tools/gpu/ab_pair.sh VARIANT...
set -e
OUT=${OUT:-gpurun_out/ab_pair}
mkdir -p "$OUT"
for v in "$@"; do
  export JANUS_PRIO3_LIB=$PWD/janus_amd/variants/libjanus_prio3_$v.so
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -k "hist" -x -q --timeout 120 --timeout-method thread > "$OUT/tests_$v.log" 2>&1 || { tail -30 "$OUT/tests_$v.log"; exit 1; }
  echo "$v: $(tail -1 $OUT/tests_$v.log)"
done
unset JANUS_PRIO3_LIB
one() {  # LIB TAG ARGS
  local lib=$1 tag=$2; shift 2
  if [ "$lib" = base ]; then unset JANUS_PRIO3_LIB; else export JANUS_PRIO3_LIB=$PWD/janus_amd/variants/libjanus_prio3_$lib.so; fi
  timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-secondary --warmup 5 --steps 40 "$@" > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail -20 "$OUT/$tag.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['value']/1e6,2), {k: round(v['ms_avg'],3) for k,v in d['kernels'].items() if v['ms_avg']>0.05}, d['checks'])"
}
for rep in 1 2; do
  one base base_h$rep --opt pair_max=0
  for v in "$@"; do one $v ${v}_p$rep --opt pair_max=2000000; done
done
