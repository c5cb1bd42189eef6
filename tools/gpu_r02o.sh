#!/bin/bash
# compiled C CPU baselines for C5 (FPVec) and mp64, with CPU/GPU parity on the sample
mkdir -p gpurun_out
T=${1:-r02o}
timeout -k 10 600 python -u -m pytest tests/test_mp64.py tests/test_fpvec.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/${T}_gpu_tests.log | head; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 600 python -u bench.py --role fpvec --steps 3 --warmup 1 > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { echo "c5 failed"; tail -20 gpurun_out/${T}_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${T}_c5.json')); print('C5', round(d['value']/1e3,1), 'K/s', d['checks'], d['cpu_baseline'])"
timeout -k 10 600 python -u bench.py --role mp64 --reports 1000000 --steps 5 --warmup 1 > gpurun_out/${T}_mp64.json 2> gpurun_out/${T}_mp64.err || { echo "mp64 failed"; tail -20 gpurun_out/${T}_mp64.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${T}_mp64.json')); print('MP64', round(d['value']/1e6,2), 'M/s', d['checks'], d['cpu_baseline'])"
