#!/bin/bash
# fuse_q=1 across chunk counts vs the default
set -e
O=gpurun_out/r02zb
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/def_$i.json
  for c in 1 2 4 8; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --opt fuse_q=1 --opt chunks=$c > $O/fq1_c${c}_$i.json
  done
done
