#!/bin/bash
# Evidence for the fused k_prep_h default: rocprofv3 passes (stats, HBM bytes, VALU, stalls),
# the default bench line (with CPU baseline), the other config lines and the jobs line.
set -e
O=gpurun_out/s3d
mkdir -p $O
SKIP_HPKE=1 bash profiles/run_profiles.sh s3d > /dev/null
timeout -k 10 300 python3 bench.py > $O/bench_c2.json
for v in count sumvec sum32; do
  timeout -k 10 200 python3 bench.py --role config --vdaf $v --no-cpu-baseline > $O/bench_$v.json
done
timeout -k 10 200 python3 bench.py --role jobs --no-cpu-baseline > $O/bench_jobs128.json
timeout -k 10 200 python3 bench.py --role leader --no-cpu-baseline > $O/bench_leader.json
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/s3d/bench_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, round(d['value']/1e6,2), d.get('ms_per_step'))
PY
