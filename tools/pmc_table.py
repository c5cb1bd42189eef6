"""Per-kernel table of the counters collected by tools/prof_query.sh (sums over dispatches,
divided by dispatch count).  Usage: python tools/pmc_table.py gpurun_out/prof_<tag> [kernel-substr]"""
import csv, glob, os, re, sys
from collections import defaultdict

src = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
vals = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(os.path.join(src, "pmc_*", "*counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        if sub not in row["Kernel_Name"]:
            continue
        m = re.search(r"(k_[A-Za-z_0-9]+)", row["Kernel_Name"])
        k = m.group(1) if m else row["Kernel_Name"][:60]
        vals[k][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[k, row["Counter_Name"]].add(row["Dispatch_Id"])
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        n = len(disp[k, c])
        print(f"  {c:24s} {v / n:16.4g}   (per dispatch, {n} dispatches)")
