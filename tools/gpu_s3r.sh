#!/bin/bash
# Leader accumulate fused into k_jrpart (leader_fuse_acc): leader parity, then the leader line A/B.
set -e
O=gpurun_out/s3r
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_leader.py tests/test_gpu_fused.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in "" "leader_fuse_acc=0" "" "leader_fuse_acc=0"; do
  opts=""; for kv in $v; do opts="$opts --opt $kv"; done
  timeout -k 10 200 python3 bench.py --role leader --no-cpu-baseline --steps 20 --warmup 3 $opts > $O/leader.json
  python3 -c "
import json; d=json.load(open('$O/leader.json')); print('[leader $v]', round(d['value']/1e6,1), round(d['ms_per_step'],4), {k: round(v['ms_avg'],4) for k,v in d.get('kernels',{}).items()}, d.get('checks'))"
done
