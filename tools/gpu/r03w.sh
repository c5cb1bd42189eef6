#!/bin/bash
# r03w: the in-kernel leader-share pull with rows loaded 4 iterations ahead (k_prep_h PULL
# at 2 waves/SIMD, 188 VGPRs): executor + fused tests, then the jobs line x3 with traces.
set -e
O=$PWD/gpurun_out/r03w
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_executor.py tests/test_gpu_fused.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in a b c; do
  JANUS_EXEC_TRACE=$O/trace_$r.txt timeout -k 10 300 python3 bench.py --role jobs --no-cpu-baseline > $O/jobs_$r.json
  python3 -c "
import json; d=json.load(open('$O/jobs_$r.json')); print('[$r]', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks']['every_job_matches_cpu'])"
done
