#!/bin/bash
# r03l: group launches with the leader-share copy issued after the XOF launch (runs under it);
# P-256 opener at 2 waves/SIMD (table in registers) vs 3 (table in private memory).
set -e
O=$PWD/gpurun_out/r03l
R=$PWD
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_executor.py tests/test_gpu_fused.py tests/test_gpu_leader.py tests/test_baseline_configs.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for mode in combined combined; do
  timeout -k 10 300 python3 bench.py --role jobs --jobs-call $mode --no-cpu-baseline > $O/jobs_$mode.json
  python3 -c "
import json; d=json.load(open('$O/jobs_$mode.json')); print('[$mode]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
done
for v in base p256w3 base p256w3; do
  if [ $v = base ]; then unset JANUS_HPKE_LIB JANUS_PRIO3_LIB; else export JANUS_PRIO3_LIB=$R/janus_amd/variants/libjanus_prio3_$v.so; fi
  timeout -k 10 200 python3 bench.py --role hpke --hpke-kem p256 --reports 262144 --steps 5 --no-cpu-baseline > $O/p256_$v.json
  python3 -c "
import json; d=json.load(open('$O/p256_$v.json')); print('[p256 $v]', round(d['value']/1e6,2), 'M/s', round(d['roofline']['frac'],3), d['checks'])"
done
unset JANUS_PRIO3_LIB
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --role jobs --no-cpu-baseline > $O/jobs_traced.json
