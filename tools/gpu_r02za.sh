#!/bin/bash
# fused accumulate in the query (fuse_q): parity, interleaved A/B, chunks=1 traces.
set -e
O=gpurun_out/r02za
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py > $O/tests.log 2>&1
for i in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --opt fuse_q=$v > $O/c2_fq${v}_$i.json
  done
done
for v in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_fq$v -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --opt chunks=1 --opt fuse_q=$v > $O/trace_fq$v.json
done
