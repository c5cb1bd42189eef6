#!/bin/bash
# r03c: k_prep_h instruction-cache and issue counters (whole-batch C2 launches), then an A/B of
# the Keccak round-loop unroll (KECCAK_UNROLL 2 = base, 1, 4).
set -e
O=$PWD/gpurun_out/r03c
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ --kernel-trace --output-format csv -d $O/pmc_ic -o run -- $B > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/pmc_sq -o run -- $B > /dev/null
cd $R
python3 tools/pmc_table.py $O k_prep_h
cd $R && STEPS=30 bash tools/ab_libs.sh base ku1 ku4 base ku1 ku4
