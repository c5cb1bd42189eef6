#!/bin/bash
# k_xof_pair: parity, then C3 / C5 lines with the lane-pair XOF on and off
mkdir -p gpurun_out
T=${1:-r02i}
timeout -k 10 900 python -u -m pytest ${PYTEST_TARGETS:-tests/test_gpu_parity.py tests/test_fpvec.py tests/test_gpu_fullsize.py} -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/${T}_gpu_tests.log | head; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
for xp in 1 0; do
  timeout -k 10 300 python -u bench.py --role config --vdaf sumvec --no-cpu-baseline --opt xof_pair=$xp > gpurun_out/${T}_c3_xp$xp.json 2> gpurun_out/${T}_c3.err || { echo "c3 failed"; tail -20 gpurun_out/${T}_c3.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_c3_xp$xp.json')); print('C3 xof_pair=$xp', round(d['value']/1e6,3), 'M/s', {k:round(v['ms_avg'],2) for k,v in d['kernels'].items() if v['ms_avg']>0.1}, d.get('checks'))"
done
for xp in 1 0; do
  timeout -k 10 400 python -u bench.py --role fpvec --steps 3 --warmup 1 --no-cpu-baseline --opt xof_pair=$xp > gpurun_out/${T}_c5_xp$xp.json 2> gpurun_out/${T}_c5.err || { echo "c5 failed"; tail -20 gpurun_out/${T}_c5.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_c5_xp$xp.json')); print('C5 xof_pair=$xp', round(d['value']/1e3,1), 'K/s', {k:round(v['ms_avg'],2) for k,v in d['kernels'].items() if v['ms_avg']>0.1}, d.get('checks'))"
done
