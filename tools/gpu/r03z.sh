#!/bin/bash
# r03z: P-256 with the w = 4 window (8-point table in private memory): HPKE tests (RFC 9180
# vectors), the P-256 hpke line; then the r03y jobs traces.
set -e
O=$PWD/gpurun_out/r03z
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hpke.py > $O/hpke_tests.log 2>&1 || { tail -30 $O/hpke_tests.log; exit 1; }
tail -1 $O/hpke_tests.log
for r in a b; do
  timeout -k 10 300 python3 bench.py --role hpke --hpke-kem p256 > $O/hpke_p256_$r.json
  python3 -c "
import json; d=json.load(open('$O/hpke_p256_$r.json')); print('[p256 $r]', round(d['value']/1e6,2), 'M/s', d.get('roofline',{}).get('frac'), d['checks'])"
done
bash tools/gpu/r03y.sh
