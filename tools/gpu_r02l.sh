#!/bin/bash
# truncation inside the XOF (SumVec under k_query_w, FPVec entry decode): parity, then C3 / C5
# with trunc_xof on and off
mkdir -p gpurun_out
T=${1:-r02l}
timeout -k 10 900 python -u -m pytest ${PYTEST_TARGETS:-tests/test_gpu_parity.py tests/test_fpvec.py} -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/${T}_gpu_tests.log | head; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
for o in "trunc_xof=1" "trunc_xof=0"; do
  f=gpurun_out/${T}_c3_${o/=/}.json
  timeout -k 10 300 python -u bench.py --role config --vdaf sumvec --no-cpu-baseline --opt $o > $f 2> gpurun_out/${T}_c3.err || { echo "c3 failed"; tail -20 gpurun_out/${T}_c3.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); print('C3 $o', round(d['value']/1e6,3), 'M/s', {k:round(v['ms_avg'],2) for k,v in d['kernels'].items() if v['ms_avg']>0.1}, d.get('checks'))"
done
for o in "trunc_xof=1" "trunc_xof=0"; do
  f=gpurun_out/${T}_c5_${o/=/}.json
  timeout -k 10 400 python -u bench.py --role fpvec --steps 3 --warmup 1 --no-cpu-baseline --opt $o > $f 2> gpurun_out/${T}_c5.err || { echo "c5 failed"; tail -20 gpurun_out/${T}_c5.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); print('C5 $o', round(d['value']/1e3,1), 'K/s', {k:round(v['ms_avg'],2) for k,v in d['kernels'].items() if v['ms_avg']>0.1}, d.get('checks'))"
done
