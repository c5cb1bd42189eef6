#!/bin/bash
# PMC passes over the C5 step (100k reports, 2 sub-batches): HBM bytes, VALU and stall counters
# for k_xof_pair and k_query_fpw.  One counter block per pass (the hardware limits).
set -e
O=gpurun_out/r02v_c5
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --role fpvec --steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- $B > /dev/null
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- $B > /dev/null
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_sq -o run -- $B > /dev/null
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 --kernel-trace --output-format csv -d $O/pmc_stall -o run -- $B > /dev/null
python3 tools/pmc_table.py $O > $O/table.txt
