#!/bin/bash
# rocprofv3 passes on the headline bench (whole-batch launches) for one engine option set:
# kernel stats, HBM bytes, VALU/wave counters, stall split, LDS counters.
# Usage (GPU box, repo root): bash tools/prof_query.sh <tag> [bench.py --opt args...]
set -e
TAG=$1; shift
R=$(pwd); OUT=$R/gpurun_out/prof_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --opt chunks=1 $@"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/bench.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- python3 $B > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- python3 $B > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc_sq -o run -- python3 $B > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $OUT/pmc_stall -o run -- python3 $B > /dev/null
echo done
