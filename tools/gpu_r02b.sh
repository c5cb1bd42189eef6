#!/bin/bash
# k_query_pair: GPU parity (whole suite), then the headline bench with the pair query on/off and
# whole-batch launches (chunks=1) for per-kernel times.
mkdir -p gpurun_out
T=${1:-r02b}
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest ${PYTEST_TARGETS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${T}_gpu_tests.log
for v in "qpair=1" "qpair=0" "qpair=1 --opt chunks=1" "qpair=0 --opt chunks=1"; do
  tag=$(echo $v | tr ' =-' '___')
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --opt $v > gpurun_out/${T}_bench_$tag.json 2> gpurun_out/${T}_bench_$tag.err \
    || { echo "bench $v failed"; tail -30 gpurun_out/${T}_bench_$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench_$tag.json')); k=d['kernels']
print('$v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms', {n:round(v['ms_avg'],3) for n,v in k.items() if v['ms_avg']>0.05})"
done
