#!/bin/bash
# k_prep_h2 (two tiles per wave, out-of-step XOF/query order by block): parity, then A/B.
set -e
O=gpurun_out/s3h
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "fused_prepare or slow_path" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SKIP_TESTS=1 STEPS=40 bash tools/ab1.sh "" "prep_lag=1" "" "prep_lag=1"
