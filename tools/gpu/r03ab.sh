#!/bin/bash
# r03ab: two launchers, the second taking the next group ~200 us before the running one is
# expected to finish (futex job waits as r03aa): executor + fused tests, jobs line x3 with traces,
# and once at one launcher; P-256 A/B.
set -e
O=$PWD/gpurun_out/r03ab
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_executor.py tests/test_gpu_fused.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in a b c; do
  JANUS_EXEC_TRACE=$O/trace_$r.txt timeout -k 10 300 python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_$r.json
  python3 -c "
import json; d=json.load(open('$O/jobs_$r.json')); print('[jobs $r]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
done
JANUS_PRIO3_MAX_INFLIGHT=1 JANUS_EXEC_TRACE=$O/trace_inf1.txt timeout -k 10 300 python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_inf1.json
python3 -c "
import json; d=json.load(open('$O/jobs_inf1.json')); print('[jobs inf1]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
# P-256: w = 4 with Z3 = 2 Y Z / 2 Z H and doublings as additions, against w = 3 (p256w3)
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hpke.py > $O/hpke_tests.log 2>&1 || { tail -30 $O/hpke_tests.log; exit 1; }
tail -1 $O/hpke_tests.log
for r in a b; do
  for v in base p256w3; do
    if [ $v = base ]; then unset JANUS_PRIO3_LIB; else export JANUS_PRIO3_LIB=$PWD/janus_amd/variants/libjanus_prio3_$v.so; fi
    timeout -k 10 300 python3 bench.py --role hpke --hpke-kem p256 --no-cpu-baseline > $O/hpke_${v}_$r.json
    python3 -c "
import json; d=json.load(open('$O/hpke_${v}_$r.json')); print('[p256 $v $r]', round(d['value']/1e6,2), 'M/s', d['checks'])"
  done
done
