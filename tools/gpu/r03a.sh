#!/bin/bash
# r03a: the BASELINE-config parity tests at bench sizes, then the whole GPU suite.
set -e
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_baseline_configs.py > $O/baseline.log 2>&1 || { tail -60 $O/baseline.log; exit 1; }
tail -8 $O/baseline.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  --durations=25 > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -30 $O/tests.log
