#!/bin/bash
# r03b: the pruned engine -- whole GPU suite, then the C2 line at 1Mi and at 5 x 3072 waves
# (983,040 reports: whole wave rounds at 3 waves/SIMD), and the available PMC counter list.
set -e
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  --durations=15 > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -18 $O/tests.log
for n in 1048576 983040 1048576 983040; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 30 --warmup 5 --reports $n > $O/c2_$n.json
  python3 -c "
import json; d=json.load(open('$O/c2_$n.json')); k=d['kernels']['k_prep_h']; print('[c2 $n]', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms/step', round(k['ms_avg'],4), 'ms k_prep_h', round(k['ms_avg']/$n*1e6,4), 'ns/report')"
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/$O/counters.txt 2>&1 || true
grep -i -E "icache|SQC_|IFETCH|INST_LEVEL|WAIT_INST" $GRAFT_REPO_ROOT/$O/counters.txt | head -40 || true
