#!/bin/bash
# The one GPU-box driver script (replaces the per-experiment one-offs of rounds 1-3).
#   OUT=gpurun_out/<tag> bash tools/gpu/run.sh STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failure ends the script.
#   tests[:K]             pytest -m gpu -x (optionally -k K)           -> $OUT/tests.log
#   testsall[:K]          the same without -x
#   smoke                 __graft_entry__.smoke()                      -> $OUT/smoke.log
#   bench:NAME[:ARGS]     python bench.py ARGS (',' separates args)    -> $OUT/NAME.json
#   lines                 every bench line (helper, configs, fpvec, leader, jobs, hpke, pipeline, mp64)
#   prof:NAME[:ARGS]      rocprofv3 --kernel-trace --stats of bench.py ARGS -> $OUT/prof_NAME/
#   pmc:NAME:CTRS[:ARGS]  one rocprofv3 --pmc pass (CTRS ','-separated) -> $OUT/pmc_NAME/
#   lib:TAG               later steps load janus_amd/variants/libjanus_prio3_TAG.so (tools/
#                         build_variant.sh; lib:base = the in-tree library again)
# e.g.  OUT=gpurun_out/r04a bash tools/gpu/run.sh tests smoke bench:c2 prof:c2:--steps,5
set -e
OUT=${OUT:-gpurun_out/run}
mkdir -p "$OUT"
export TMPDIR=/tmp
args() { echo "${1//,/ }"; }
summ() {  # one line per bench json: value, ms/step, roofline frac, cpu baseline, boolean checks
  python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
cb = d.get("cpu_baseline") or {}
rf = d.get("roofline") or {}
ck = d.get("checks") or {}
print(sys.argv[1].split("/")[-1], round(d["value"] / 1e6, 3), "M", d.get("unit"), "ms",
      round(d.get("ms_per_step") or 0, 4), "frac", rf.get("frac"), "cpu", cb.get("value"),
      {k: v for k, v in ck.items() if isinstance(v, bool)})
for k, v in d.items():
    if k.startswith("secondary_") and isinstance(v, dict):
        print(" ", k, round((v.get("value") or 0) / 1e6, 3), "M ms", round(v.get("ms_per_step") or 0, 4),
              "frac", (v.get("roofline") or {}).get("frac"), v.get("error", ""),
              {c: x for c, x in (v.get("checks") or {}).items() if isinstance(x, bool)})
if "secondary_seconds" in d:
    print("  secondary_seconds", round(d["secondary_seconds"], 1))
PY
}
bench() {  # NAME ARGS...
  local name=$1; shift
  local t0=$SECONDS
  timeout -k 10 600 python3 bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  echo "$name wall $((SECONDS - t0)) s"
  summ "$OUT/$name.json"
}
for step in "$@"; do
  IFS=: read -r kind a1 a2 a3 <<< "$step"
  case $kind in
  tests|testsall)  # testsall: no -x, every selected test runs (a failure still ends the script)
    K=(); [ -n "$a1" ] && K=(-k "$a1")
    X=(-x); [ "$kind" = testsall ] && X=()
    timeout -k 10 900 python3 -u -m pytest tests -m gpu "${X[@]}" -v --timeout 180 --timeout-method thread "${K[@]}" > "$OUT/tests.log" 2>&1 || { grep -E "FAILED|passed|failed" "$OUT/tests.log" | tail -30; exit 1; }
    tail -1 "$OUT/tests.log" ;;
  probe)  # the driver's process / queue limits the 8-rank test depends on
    { for f in hws_max_conc_proc sched_policy hws_gws_support mes cwsr_enable; do
        echo "amdgpu.$f = $(cat /sys/module/amdgpu/parameters/$f 2>&1)"; done
      for n in /sys/class/kfd/kfd/topology/nodes/*/properties; do
        grep -E "^(simd_count|cpu_cores_count|num_cp_queues|num_sdma_engines|num_sdma_xgmi_engines|num_sdma_queues_per_engine|max_waves_per_simd|gfx_target_version|num_xcc)" "$n" | tr '\n' ' '; echo " <- $n"; done
      ls -l /proc/self/fd 2>&1 | grep -c kfd || true
    } > "$OUT/probe.txt" 2>&1; cat "$OUT/probe.txt" ;;
  smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
    tail -1 "$OUT/smoke.log" ;;
  bench)
    bench "$a1" $(args "$a2") ;;
  lines)
    bench c2
    bench c1 --role config --vdaf count
    bench c3 --role config --vdaf sumvec
    bench c4 --role config --vdaf sum32
    bench c5 --role fpvec
    bench leader --role leader
    bench leader_sum32 --role leader --leader-vdaf sum32
    bench jobs128 --role jobs
    bench hpke --role hpke --reports 1048576
    bench hpke_p256 --role hpke --hpke-kem p256 --reports 262144
    bench hpke_x448 --role hpke --hpke-kem x448 --reports 262144
    bench hpke_p521 --role hpke --hpke-kem p521 --reports 262144
    bench hpke_p384 --role hpke --hpke-kem p384 --reports 65536
    bench pipeline --role pipeline --reports 1048576
    bench mp64 --role mp64 --reports 1000000 ;;
  prof)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$a1" -o run -- python3 bench.py --no-cpu-baseline --no-secondary $(args "$a2") > "$OUT/prof_$a1.json" 2> "$OUT/prof_$a1.err" || { tail -20 "$OUT/prof_$a1.err"; exit 1; }
    summ "$OUT/prof_$a1.json" ;;
  pmc)
    timeout -s KILL 120 rocprofv3 --pmc $(args "$a2") --output-format csv -d "$OUT/pmc_$a1" -o run -- python3 bench.py --no-cpu-baseline --no-secondary --warmup 1 --steps 2 $(args "$a3") > "$OUT/pmc_$a1.json" 2> "$OUT/pmc_$a1.err" || { tail -20 "$OUT/pmc_$a1.err"; exit 1; }
    echo "pmc $a1 done" ;;
  lib)
    if [ "$a1" = base ]; then unset JANUS_PRIO3_LIB; else export JANUS_PRIO3_LIB=$PWD/janus_amd/variants/libjanus_prio3_$a1.so; fi
    echo "lib $a1" ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
