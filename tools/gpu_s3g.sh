#!/bin/bash
# DHKEM(P-256, HKDF-SHA256): HPKE GPU tests, then the hpke line for P-256 x {AES-128-GCM, ChaCha}.
set -e
O=gpurun_out/s3g
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_hpke.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for a in 1 3; do
  timeout -k 10 200 python3 bench.py --role hpke --hpke-kem p256 --hpke-aead $a --reports 262144 > $O/hpke_p256_$a.json
  python3 -c "
import json; d=json.load(open('$O/hpke_p256_$a.json')); print(d['metric'], round(d['value']/1e6,2), d['kernel_ms_avg'], d.get('cpu_baseline',{}).get('value'), d['checks'])"
done
