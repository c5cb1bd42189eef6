set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1_tests.log 2>&1 || { tail -20 gpurun_out/ab1_tests.log; exit 1; }
tail -2 gpurun_out/ab1_tests.log
for v in "qh_prefetch=0 --opt qh_occ=3" "qh_prefetch=1 --opt qh_occ=3" "qh_prefetch=0 --opt qh_occ=2" "qh_prefetch=1 --opt qh_occ=2"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --opt $v > gpurun_out/ab1.json
  python -c "
import json; d=json.load(open('gpurun_out/ab1.json')); print('$v', round(d['value']/1e6,2), {k: round(v['ms_avg'],3) for k,v in d['kernels'].items() if v['ms_avg']>0.05})"
done
