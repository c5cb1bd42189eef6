#!/bin/bash
# Cost of the fused accumulate inside k_xofd: chunks=1 traces with fuse_acc 1 and 0.
set -e
O=gpurun_out/r02z
mkdir -p $O
export TMPDIR=/tmp
for f in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_f$f -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --opt chunks=1 --opt fuse_acc=$f > $O/trace_f$f.json
done
