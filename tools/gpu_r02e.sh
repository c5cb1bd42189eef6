#!/bin/bash
# Workspace / executor refactor: full GPU suite, then the headline bench.
mkdir -p gpurun_out
T=${1:-r02e}
timeout -k 10 900 python -u -m pytest ${PYTEST_TARGETS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|error" gpurun_out/${T}_gpu_tests.log | head -20; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { echo "bench failed"; tail -30 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms', d['checks'])"
timeout -k 10 300 python -u bench.py --role jobs --no-cpu-baseline > gpurun_out/${T}_jobs.json 2> gpurun_out/${T}_jobs.err \
  || { echo "jobs bench failed"; tail -30 gpurun_out/${T}_jobs.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${T}_jobs.json')); print('jobs', round(d['value']/1e6,2), 'M/s', d['coalescing'], d['checks'], d['pcie'])"
