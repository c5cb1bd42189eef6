#!/bin/bash
# Round-2 first GPU session: full GPU test suite, the FPVec r01u geometry under the device-check
# build (ld 86016 > sub 50176, ld_out 100032, 100k x 10000), and the default bench line.
mkdir -p gpurun_out
T=${1:-r02a}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${T}_gpu_tests.log
JANUS_PRIO3_LIB=janus_amd/libjanus_prio3_dbg.so timeout -k 10 300 python -u bench.py --role fpvec \
  --steps 2 --warmup 1 --no-cpu-baseline --opt fp_sub_bytes=225460000000 \
  > gpurun_out/${T}_fpvec_dbg_r01u_geometry.json 2> gpurun_out/${T}_fpvec_dbg.err \
  || { echo "fpvec dbg failed"; tail -30 gpurun_out/${T}_fpvec_dbg.err; exit 1; }
cat gpurun_out/${T}_fpvec_dbg_r01u_geometry.json
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { echo "bench failed"; tail -30 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
