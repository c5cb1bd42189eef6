#!/bin/bash
# r03h: the tail-free dual-state share loop + four 8-point Lagrange phases (variant v1): whole GPU
# suite on v1, then an interleaved C2 A/B against the current build.
set -e
O=gpurun_out/r03h
mkdir -p $O
JANUS_PRIO3_LIB=$PWD/janus_amd/variants/libjanus_prio3_v1.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_v1.log 2>&1 || { tail -40 $O/tests_v1.log; exit 1; }
tail -1 $O/tests_v1.log
STEPS=30 bash tools/ab_libs.sh base v1 base v1 base v1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist.py > $O/dist.log 2>&1 || { tail -40 $O/dist.log; exit 1; }
tail -1 $O/dist.log
