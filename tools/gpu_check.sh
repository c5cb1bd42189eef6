#!/bin/bash
# One GPU-box session: parity tests, the default bench line, then the rocprofv3 evidence.
# Usage (from the repo root, on the GPU box): bash tools/gpu_check.sh <tag>
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 python -u bench.py --role hpke > gpurun_out/bench_hpke_$TAG.json 2> gpurun_out/bench_hpke_$TAG.err || { echo "hpke bench failed"; tail -30 gpurun_out/bench_hpke_$TAG.err; exit 1; }
cat gpurun_out/bench_hpke_$TAG.json
timeout -k 10 400 python -u bench.py --role pipeline > gpurun_out/bench_pipeline_$TAG.json 2> gpurun_out/bench_pipeline_$TAG.err || { echo "pipeline bench failed"; tail -30 gpurun_out/bench_pipeline_$TAG.err; exit 1; }
cat gpurun_out/bench_pipeline_$TAG.json
bash profiles/run_profiles.sh $TAG
