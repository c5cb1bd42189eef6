#!/bin/bash
# Round-3 end evidence (c, after the P-256 w = 4 window and the executor's output copy kernel):
# the whole GPU suite, smoke(), and every bench line with its CPU baseline and CPU/GPU parity on
# the sample, into gpurun_out/final3c/; then the P-256 line's issued-instruction pass.
set -e
O=gpurun_out/final3c
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
# the issued-instruction row of the P-256 line (SQ_INSTS_VALU pass)
export ISSUED_TABLE=$PWD/gpurun_out/final3c_issued.json TMPDIR=/tmp
R=$PWD
P=$PWD/gpurun_out/final3c/pmc
mkdir -p $P
(cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $P/pmc_hpke_p256_aead1 -o run -- python3 $R/bench.py --role hpke --hpke-kem p256 --reports 262144 --steps 1 --warmup 0 --no-cpu-baseline > $P/pmc_hpke_p256_aead1.json)
python3 tools/pmc_issued.py hpke_p256_aead1 $P/pmc_hpke_p256_aead1 $P/pmc_hpke_p256_aead1.json --kernels k_hpke_open
