#!/bin/bash
# Prio3Sum query kernel: parity, then C4 A/B (generic k_query vs k_query_sum at 3 and 2 waves)
# and a chunks=1 kernel trace of each.
set -e
O=gpurun_out/r02x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "sum" tests/test_gpu_fused.py -k "sum" > $O/tests.log 2>&1
B="python3 bench.py --role config --vdaf sum32 --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 200 $B --opt qsum=0 > $O/c4_generic_$i.json
  timeout -k 10 200 $B --opt qsum=1 --opt qsum_occ=3 > $O/c4_occ3_$i.json
  timeout -k 10 200 $B --opt qsum=1 --opt qsum_occ=2 > $O/c4_occ2_$i.json
done
for v in "0 3" "1 3" "1 2"; do
  set -- $v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_q$1_o$2 -o run -- \
    python3 bench.py --role config --vdaf sum32 --steps 3 --warmup 1 --no-cpu-baseline --opt chunks=1 --opt qsum=$1 --opt qsum_occ=$2 > $O/trace_q$1_o$2.json
done
