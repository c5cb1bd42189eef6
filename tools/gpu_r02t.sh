#!/bin/bash
# P = 32 eight-lane query (qwide32): parity, then an interleaved A/B on the headline and a
# chunks=1 kernel trace of each.
set -e
O=gpurun_out/r02t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "p32 or wide or comparison" tests/test_gpu_fused.py > $O/tests.log 2>&1
# variants: a = k_query_h (round 2), b = + msg_cmp, c = eight-lane P=32 + msg_cmp
A="--opt qwide32=0 --opt msg_cmp=0"; B="--opt qwide32=0 --opt msg_cmp=1"; C="--opt qwide32=1 --opt msg_cmp=1"
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline $A > $O/c2_a_$i.json
  timeout -k 10 200 python3 bench.py --no-cpu-baseline $B > $O/c2_b_$i.json
  timeout -k 10 200 python3 bench.py --no-cpu-baseline $C > $O/c2_c_$i.json
done
for v in a b c; do
  case $v in a) X=$A;; b) X=$B;; c) X=$C;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --opt chunks=1 $X > $O/trace_$v.json
done
