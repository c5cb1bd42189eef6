#!/bin/bash
# Round-3 end evidence (a): the whole GPU suite, smoke(), and every bench line with its CPU
# baseline and CPU/GPU parity on the sample, into gpurun_out/final3/.
set -e
O=gpurun_out/final3
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
line() { local K=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $O/$K.json; python3 - "$O/$K.json" "$K" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
cb = d.get("cpu_baseline") or {}
r = d.get("roofline") or {}
ch = d.get("checks", {})
print(sys.argv[2], round(d["value"] / 1e6, 3), "M/s", "frac", r.get("frac") and round(r["frac"], 3),
      "cpu", cb.get("value") and round(cb["value"]), "parity", ch.get("cpu_gpu_parity_on_sample", ch.get("every_job_matches_cpu")))
PY
}
line c2
line c1 --role config --vdaf count
line c3 --role config --vdaf sumvec
line c4 --role config --vdaf sum32
line c5 --role fpvec
line leader --role leader
line leader_sum32 --role leader --leader-vdaf sum32
line jobs128 --role jobs
line hpke --role hpke --reports 1048576
line hpke_p256 --role hpke --hpke-kem p256 --reports 262144
line pipeline --role pipeline --reports 1048576
line mp64 --role mp64 --reports 1000000
