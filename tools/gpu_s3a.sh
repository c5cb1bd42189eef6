#!/bin/bash
# Session-3 A/B: cost of the per-chunk k_xof_slow launch (variant without it), a kernel trace of
# the default chunked step, and C5 in 3 sub-batches (one XOF wave per SIMD) vs the default 2.
set -e
O=gpurun_out/s3a
mkdir -p $O
STEPS=40 bash tools/ab_libs.sh base noslow base noslow > $O/ab_noslow.txt 2>&1
cat $O/ab_noslow.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/trace -o c2 --output-format csv -- python3 bench.py --no-cpu-baseline --warmup 3 --steps 5 > $O/trace_bench.json
for v in "" "fp_sub_bytes=105000000000" ""  "fp_sub_bytes=105000000000"; do
  opts=""; for kv in $v; do opts="$opts --opt $kv"; done
  timeout -k 10 300 python3 bench.py --role fpvec --no-cpu-baseline --steps 3 --warmup 1 $opts > $O/c5.json
  python3 -c "
import json; d=json.load(open('$O/c5.json')); print('[c5 $v]', round(d['value'],1), {k: round(v['ms_avg'],2) for k,v in d.get('kernels',{}).items() if v.get('ms_avg',0)>0.05})"
done
