#!/bin/bash
# FPVec sub-batches rounded to whole query rounds (fp_round): parity, then C5 A/B.
set -e
O=gpurun_out/r02zd
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_fpvec.py > $O/tests.log 2>&1
for i in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 python3 bench.py --role fpvec --no-cpu-baseline --opt fp_round=$v > $O/c5_r${v}_$i.json
  done
done
