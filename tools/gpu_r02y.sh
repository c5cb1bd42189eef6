#!/bin/bash
# k_query_sum with blocked-MAC p(t): parity, C4 at 3 and 2 waves, chunks=1 traces.
set -e
O=gpurun_out/r02y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "query_sum" > $O/tests.log 2>&1
B="python3 bench.py --role config --vdaf sum32 --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 200 $B --opt qsum_occ=3 > $O/c4_occ3_$i.json
  timeout -k 10 200 $B --opt qsum_occ=2 > $O/c4_occ2_$i.json
done
for o in 3 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_o$o -o run -- \
    python3 bench.py --role config --vdaf sum32 --steps 3 --warmup 1 --no-cpu-baseline --opt chunks=1 --opt qsum_occ=$o > $O/trace_o$o.json
done
