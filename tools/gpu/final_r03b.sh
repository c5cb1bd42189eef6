#!/bin/bash
# Round-3 end evidence (b): the C2 kernel trace and PMC passes (profiles/run_profiles.sh) and the
# issued-instruction table's C2 row for the final code.
set -e
SKIP_HPKE=1 bash profiles/run_profiles.sh r03final
export ISSUED_TABLE=$PWD/gpurun_out/final3b_issued.json TMPDIR=/tmp
R=$PWD
O=$PWD/gpurun_out/final3b
mkdir -p $O
line() {
  local K=$1; shift
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $O/pmc_$K -o run -- python3 $R/bench.py "$@" --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_$K.json)
  python3 tools/pmc_issued.py $K $O/pmc_$K $O/pmc_$K.json "${EXTRA[@]}"
}
EXTRA=(); line c2
EXTRA=(--kernels k_hpke_open); line hpke_p256_aead1 --role hpke --hpke-kem p256 --reports 262144
