#!/bin/bash
# k_query_rows: parity (the new row-split tests + the fused/parity suites), A/B against k_query_h,
# then rocprof passes (trace/stats, HBM bytes, VALU) of whole-batch launches for both.
set -e
O=gpurun_out/s3b
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_golden.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SKIP_TESTS=1 STEPS=40 bash tools/ab1.sh "qrows=1" "qrows=0" "qrows=1" "qrows=0"
bash tools/prof_query.sh s3b_rows --opt qrows=1 > /dev/null
bash tools/prof_query.sh s3b_qh --opt qrows=0 > /dev/null
python3 tools/pmc_table.py gpurun_out/prof_s3b_rows k_query > $O/pmc_rows.txt; python3 tools/pmc_table.py gpurun_out/prof_s3b_qh k_query > $O/pmc_qh.txt; cat $O/pmc_rows.txt $O/pmc_qh.txt
