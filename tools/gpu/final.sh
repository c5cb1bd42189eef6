#!/bin/bash
# Round-end evidence: whole GPU suite, smoke(), and every bench line (each with its CPU baseline
# and CPU/GPU parity on the sample), written to gpurun_out/final/.
set -e
O=gpurun_out/final
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/c2.json
timeout -k 10 200 python3 bench.py --role config --vdaf count > $O/c1.json
timeout -k 10 300 python3 bench.py --role config --vdaf sumvec > $O/c3.json
timeout -k 10 200 python3 bench.py --role config --vdaf sum32 > $O/c4.json
timeout -k 10 400 python3 bench.py --role fpvec > $O/c5.json
timeout -k 10 200 python3 bench.py --role leader > $O/leader.json
timeout -k 10 200 python3 bench.py --role leader --leader-vdaf sum32 > $O/leader_sum32.json
timeout -k 10 200 python3 bench.py --role jobs > $O/jobs128.json
timeout -k 10 200 python3 bench.py --role hpke --reports 1048576 > $O/hpke.json
timeout -k 10 200 python3 bench.py --role hpke --hpke-kem p256 --reports 262144 > $O/hpke_p256.json
timeout -k 10 200 python3 bench.py --role pipeline --reports 1048576 > $O/pipeline.json
timeout -k 10 200 python3 bench.py --role mp64 --reports 1000000 > $O/mp64.json
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/final/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    cb = d.get("cpu_baseline") or {}
    print(f.split("/")[-1], round(d["value"], 1), round(d.get("ms_per_step") or 0, 4), cb.get("value"), d.get("checks", {}).get("cpu_gpu_parity_on_sample"))
PY
