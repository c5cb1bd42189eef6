#!/bin/bash
# Prio3Sum leader on k_query_sum: parity, then the leader line for Sum(32) (new vs generic) and
# the Histogram leader line.
set -e
O=gpurun_out/r02zc
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_leader.py > $O/tests.log 2>&1
timeout -k 10 300 python3 bench.py --role leader --leader-vdaf sum32 > $O/leader_sum32.json
timeout -k 10 300 python3 bench.py --role leader --leader-vdaf sum32 --no-cpu-baseline --opt qsum=0 > $O/leader_sum32_generic.json
timeout -k 10 300 python3 bench.py --role leader > $O/leader_hist.json
