"""Issued VALU lane-instructions per report of one bench.py line, from a rocprofv3 PMC pass
(SQ_INSTS_VALU, wave-instructions per dispatch) over the same command, written into the
committed table profiles/issued_per_report.json that bench.py's model_roofline reads.

  issued = sum over the step's kernels k of  mean SQ_INSTS_VALU(k) per dispatch
                                            x launches of k per step (bench JSON `kernels`)
                                            x 64 lanes / reports per step

Usage: python tools/pmc_issued.py <line-key> <pmc dir> <bench json> [--kernels k1,k2]
(--kernels: for lines whose JSON has no per-kernel launch table, e.g. hpke: one launch each)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.environ.get("ISSUED_TABLE") or os.path.join(ROOT, "profiles", "issued_per_report.json")


def main():
    key, pmc_dir, bench_json = sys.argv[1:4]
    only = None
    if "--kernels" in sys.argv:
        only = sys.argv[sys.argv.index("--kernels") + 1].split(",")
    d = json.loads(open(bench_json).read().strip().splitlines()[-1])
    n = d["config"].get("reports_per_gpu") or d["config"].get("reports") or d["config"].get("job_size")
    steps = d["steps"]
    if only:
        per_step = {k: 1.0 for k in only}
    else:
        kt = d.get("kernels_timed_region") or d.get("kernels", {})
        per_step = {k: v["launches"] / steps for k, v in kt.items() if v.get("launches")}
    tot, disp = defaultdict(float), defaultdict(set)
    for f in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != "SQ_INSTS_VALU":
                continue
            m = re.search(r"\b(k_[A-Za-z_0-9]+)(<[^>]*>)?", row["Kernel_Name"])
            if not m:
                continue
            # a --kernels entry may name one instantiation (k_mp64_prepare<0>)
            name = m.group(1) + (m.group(2) or "")
            if name not in per_step:
                name = m.group(1)
                if name not in per_step:
                    continue
            tot[name] += float(row["Counter_Value"])
            disp[name].add(row["Dispatch_Id"])
    parts = {k: tot[k] / len(disp[k]) * per_step[k] * 64 / n for k in tot}
    table = json.load(open(TABLE)) if os.path.exists(TABLE) else {}
    table[key] = dict(issued_instr_per_report=sum(parts.values()),
                      per_kernel={k: round(v, 1) for k, v in parts.items()},
                      reports=n, source=os.path.relpath(pmc_dir, ROOT))
    json.dump(table, open(TABLE, "w"), indent=1, sort_keys=True)
    print(key, round(sum(parts.values())), {k: round(v) for k, v in parts.items()})


if __name__ == "__main__":
    main()
