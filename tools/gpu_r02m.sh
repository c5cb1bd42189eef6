#!/bin/bash
# eight-lane FPVec query (k_query_fpw): parity, then C5 with fp_wide / fp_wgs / trunc_xof A/B
mkdir -p gpurun_out
T=${1:-r02m}
timeout -k 10 900 python -u -m pytest ${PYTEST_TARGETS:-tests/test_fpvec.py} -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/${T}_gpu_tests.log | head; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
for o in "fp_wgs=3" "fp_wgs=4" "fp_wgs=2" "trunc_xof=0"; do
  f=gpurun_out/${T}_c5_${o/=/}.json
  timeout -k 10 400 python -u bench.py --role fpvec --steps 3 --warmup 1 --no-cpu-baseline --opt $o > $f 2> gpurun_out/${T}_c5.err || { echo "c5 failed"; tail -20 gpurun_out/${T}_c5.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); print('C5 $o', round(d['value']/1e3,1), 'K/s', {k:round(v['ms_avg'],2) for k,v in d['kernels'].items() if v['ms_avg']>0.1}, d.get('checks'))"
done
