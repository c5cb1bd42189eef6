#!/bin/bash
# Tail kernels: k_meta grid-stride tiles (block-level running partials), k_agg_waves 16-byte
# loads -- fused/metadata/dist parity, then the headline bench twice.
set -e
O=gpurun_out/s3f
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_batch_metadata.py tests/test_gpu_dist.py tests/test_gpu_golden.py \
  tests/test_gpu_edges.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SKIP_TESTS=1 STEPS=40 bash tools/ab1.sh "" ""
