#!/bin/bash
# P-256 fixed signed window + dedicated squaring: HPKE parity, then the P-256 HPKE line.
set -e
O=gpurun_out/s3o
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_hpke.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for a in 1 3; do
  timeout -k 10 300 python3 bench.py --role hpke --hpke-kem p256 --hpke-aead $a --reports 262144 --steps 10 --warmup 2 > $O/hpke_p256_a$a.json
  python3 -c "
import json; d=json.load(open('$O/hpke_p256_a$a.json')); print('[p256 aead $a]', round(d['value']/1e6,2), round(d['ms_per_step'],3), (d.get('roofline') or {}).get('frac'), d.get('checks'))"
done
