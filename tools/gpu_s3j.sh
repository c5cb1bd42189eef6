#!/bin/bash
# Final-state evidence: the whole GPU suite, smoke(), the default bench line (with CPU baseline),
# the rocprofv3 passes of the default step (helper + hpke), and the C5 line.
set -e
O=gpurun_out/s3j
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench_c2.json
bash profiles/run_profiles.sh s3j > /dev/null
timeout -k 10 400 python3 bench.py --role fpvec > $O/bench_c5.json
python3 - <<'PY'
import json
for f in ["gpurun_out/s3j/bench_c2.json", "gpurun_out/s3j/bench_c5.json"]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"], 1), d.get("ms_per_step"), d["checks"])
PY
