#!/bin/bash
# refresh every bench line on the current code (round-2 numbers for README / DESIGN)
mkdir -p gpurun_out
T=${1:-r02p}
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${T}_${name}.json 2> gpurun_out/${T}_${name}.err || { echo "$name failed"; tail -20 gpurun_out/${T}_${name}.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_${name}.json')); c=d.get('cpu_baseline') or {}; print('$name', round(d['value']/1e6,3), 'M/s', 'cpu', c.get('value'), d.get('checks'))"
}
run c2 && run leader --role leader && run hpke --role hpke && run pipeline --role pipeline && \
run c1 --role config --vdaf count && run c3 --role config --vdaf sumvec && run c4 --role config --vdaf sum32 && \
run jobs128 --role jobs --threads 128 && run jobs16 --role jobs --threads 16
