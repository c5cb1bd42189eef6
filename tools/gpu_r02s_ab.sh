#!/bin/bash
# A/B of the k_xof_slow geometry (slow_rpl 16 vs the round-1 one-report-per-lane grid),
# interleaved, then a chunks=1 kernel trace of each.
set -e
O=gpurun_out/r02s_ab
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for v in 16 1; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --opt slow_rpl=$v > $O/c2_rpl${v}_$i.json
  done
done
for v in 16 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_rpl$v -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --opt chunks=1 --opt slow_rpl=$v > $O/trace_rpl$v.json
done
