# GPU A/B helper: field self-test + parity suite, then bench variants given as arguments
# (each argument is one space-separated list of --opt key=value settings; "" = defaults).
set -e
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/test_field_asm.py tests/test_gpu_fused.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1_tests.log 2>&1 || { tail -30 gpurun_out/ab1_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/ab1_tests.log
for v in "$@"; do
  opts=""; for kv in $v; do opts="$opts --opt $kv"; done
  timeout -k 10 120 python bench.py --no-cpu-baseline --warmup 5 --steps ${STEPS:-40} $opts > gpurun_out/ab1.json
  python -c "
import json; d=json.load(open('gpurun_out/ab1.json')); print('[$v]', round(d['value']/1e6,2), {k: round(v['ms_avg'],3) for k,v in d['kernels'].items() if v['ms_avg']>0.05})"
done
