#!/bin/bash
# Fused k_prep_h (XOF + query in one launch, slow path inside the query): parity, then an
# interleaved A/B against the two-kernel chain with and without the k_xof_slow launch.
set -e
O=gpurun_out/s3c
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/ \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SKIP_TESTS=1 STEPS=40 bash tools/ab1.sh "" "prep_persist=1" "prep_fused=0" "prep_fused=0 slow_defer=0" "" "prep_persist=1" "prep_fused=0" "chunks=8"
