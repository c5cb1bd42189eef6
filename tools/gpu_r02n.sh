#!/bin/bash
# DAP decode semantics, roctx ranges, headline bench with the aggregate CPU/GPU parity check
mkdir -p gpurun_out
T=${1:-r02n}
timeout -k 10 900 python -u -m pytest tests/test_dap_codec.py tests/test_gpu_pipeline.py tests/test_gpu_executor.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/${T}_gpu_tests.log | head; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('C2', round(d['value']/1e6,2), 'M/s', d['checks'], d['cpu_baseline']['value'])"
