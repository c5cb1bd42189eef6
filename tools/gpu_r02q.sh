#!/bin/bash
# FPVec leader role on the device + regressions of the leader / e2e / FPVec suites
mkdir -p gpurun_out
T=${1:-r02q}
timeout -k 10 900 python -u -m pytest tests/test_fpvec.py tests/test_reference_e2e.py tests/test_gpu_leader.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|assert" gpurun_out/${T}_gpu_tests.log | head -20; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
