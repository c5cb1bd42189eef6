#!/bin/bash
# Collects the rocprofv3 evidence for bench.py (run on the GPU box from the repo root).
# Usage: bash profiles/run_profiles.sh <tag> [extra bench.py args for the helper role]
# The helper passes run whole-batch launches (--opt chunks=1), matching the isolated roofline
# pass bench.py reports (the default bench cuts the batch into 8 stream-overlapped chunks).
set -e
TAG=${1:-r01}
shift || true
EXTRA="${@:---opt chunks=1}"
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp

passes() {  # $1 = subdirectory prefix, rest = bench.py arguments
  local P=$1
  shift
  # 1) kernel trace + stats on the benchmark command itself
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${P}trace -o run -- \
    python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary "$@" > $OUT/${P}bench_under_trace.json
  # 2) HBM traffic counters, one block per pass (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2)
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/${P}pmc_fetch -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary "$@" > /dev/null
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/${P}pmc_write -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary "$@" > /dev/null
  # 3) VALU / wave occupancy counters
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/${P}pmc_sq -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary "$@" > /dev/null
  # 4) where the wave cycles go (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES)
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 --kernel-trace --output-format csv -d $OUT/${P}pmc_stall -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary "$@" > /dev/null
}

passes "" $EXTRA
[ -n "$SKIP_HPKE" ] || passes "hpke_" --role hpke --reports 262144
ls $OUT
