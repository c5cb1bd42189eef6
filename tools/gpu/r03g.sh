#!/bin/bash
# r03g: session start on the re-created container -- whole GPU suite, smoke(), the C2 line and its
# kernel trace.
set -e
O=$PWD/gpurun_out/r03g
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/c2.json
python3 -c "import json; d=json.load(open('$O/c2.json')); print(round(d['value']/1e6,2), d['roofline'], d['cpu_baseline'], d['checks'])"
export TMPDIR=/tmp
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --opt chunks=1 > $O/c2_traced.json
ls $O/trace/*/
