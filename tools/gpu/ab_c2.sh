#!/bin/bash
# Interleaved A/B of the headline step (C2) between the in-tree library and variants, after the
# Histogram parity tests on the in-tree build:  OUT=... bash tools/gpu/ab_c2.sh "VARIANTS" REPS
set -e
OUT=${OUT:-gpurun_out/ab_c2}
mkdir -p "$OUT"
VARS=$1; REPS=${2:-3}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_leader.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
echo "tests: $(tail -1 $OUT/tests.log)"
for rep in $(seq $REPS); do
  for v in base $VARS; do
    if [ "$v" = base ]; then unset JANUS_PRIO3_LIB; else export JANUS_PRIO3_LIB=$PWD/janus_amd/variants/libjanus_prio3_$v.so; fi
    timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-secondary --warmup 5 --steps 40 > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || { tail -20 "$OUT/${v}_$rep.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); print('$v $rep', round(d['value']/1e6,2), {k: round(x['ms_avg'],3) for k,x in d['kernels'].items() if x['ms_avg']>0.05})"
  done
done
