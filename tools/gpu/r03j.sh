#!/bin/bash
# r03j: every bench line once with its model roofline, and a SQ_INSTS_VALU pass of each for the
# issued-instruction table (tools/pmc_issued.py); then the fused kernel vs the two-kernel chain at
# a jobs-sized batch (32k reports).
set -e
O=$PWD/gpurun_out/r03j
R=$PWD
mkdir -p $O
export ISSUED_TABLE=$O/issued_per_report.json TMPDIR=/tmp
line() {  # key, bench args...
  local K=$1; shift
  timeout -k 10 300 python3 $R/bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline > $O/$K.json
  python3 -c "
import json; d=json.load(open('$O/$K.json')); r=d.get('roofline') or {}; print('$K', round(d['value']/1e6,3), 'M/s frac', r.get('frac'))"
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $O/pmc_$K -o run -- python3 $R/bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_$K.json)
}
line c2
python3 tools/pmc_issued.py c2 $O/pmc_c2 $O/pmc_c2.json
line config_count --role config --vdaf count
python3 tools/pmc_issued.py config_count $O/pmc_config_count $O/pmc_config_count.json
line config_sumvec --role config --vdaf sumvec
python3 tools/pmc_issued.py config_sumvec $O/pmc_config_sumvec $O/pmc_config_sumvec.json
line config_sum32 --role config --vdaf sum32
python3 tools/pmc_issued.py config_sum32 $O/pmc_config_sum32 $O/pmc_config_sum32.json
line leader_hist --role leader
python3 tools/pmc_issued.py leader_hist $O/pmc_leader_hist $O/pmc_leader_hist.json
line leader_sum32 --role leader --leader-vdaf sum32
python3 tools/pmc_issued.py leader_sum32 $O/pmc_leader_sum32 $O/pmc_leader_sum32.json
line hpke_x25519_aead1 --role hpke --reports 262144
python3 tools/pmc_issued.py hpke_x25519_aead1 $O/pmc_hpke_x25519_aead1 $O/pmc_hpke_x25519_aead1.json --kernels k_hpke_open
line hpke_p256_aead1 --role hpke --hpke-kem p256 --reports 262144
python3 tools/pmc_issued.py hpke_p256_aead1 $O/pmc_hpke_p256_aead1 $O/pmc_hpke_p256_aead1.json --kernels k_hpke_open
line mp64 --role mp64 --reports 262144
python3 tools/pmc_issued.py mp64 $O/pmc_mp64 $O/pmc_mp64.json
line fpvec --role fpvec
python3 tools/pmc_issued.py fpvec $O/pmc_fpvec $O/pmc_fpvec.json
for v in base split base split; do
  if [ $v = base ]; then unset JANUS_PRIO3_LIB; else export JANUS_PRIO3_LIB=$R/janus_amd/variants/libjanus_prio3_$v.so; fi
  timeout -k 10 120 python3 bench.py --reports 32768 --steps 30 --warmup 3 --no-cpu-baseline > $O/ab32k_$v.json
  python3 -c "
import json; d=json.load(open('$O/ab32k_$v.json')); print('[$v 32k]', round(d['value']/1e6,2), {k: round(v['ms_avg'],3) for k,v in d['kernels'].items()})"
done
