"""Summarise the rocprofv3 output of profiles/run_profiles.sh into committed evidence.

Usage: python tools/summarize_profiles.py gpurun_out/prof_<tag> <tag>

Writes
  profiles/<tag>_rocprof_summary.txt  kernel-trace stats (avg duration per kernel), HBM bytes per
                                      launch from the FETCH_SIZE / WRITE_SIZE passes, SQ counters;
  profiles/kernel_counts.json         per kernel: HBM bytes per launch, dynamic VALU instructions
                                      per work-item (SQ_INSTS_VALU / SQ_WAVES; one report per
                                      lane), and the mix-weighted VALU ceiling of its hottest
                                      loop (tools/isa_mix.py).  bench.py reads it for `roofline`.

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md ("HBM [CDNA4]"): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced
streaming read, so it is doubled; WRITE_SIZE is taken as is.
"""
from __future__ import annotations

import csv
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    m = re.match(r"(?:void )?([A-Za-z_0-9]+)(<[^(]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def counters(path):
    """kernel short name -> counter -> list of per-dispatch values."""
    out = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return out
    with open(path) as f:
        for row in csv.DictReader(f):
            out[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return out


def main():
    src, tag = sys.argv[1], sys.argv[2]
    lines = [f"# rocprofv3 summary, tag {tag} (source: {src}, produced by profiles/run_profiles.sh)",
             "# commands: python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --opt chunks=1 "
             "(Prio3Histogram(256,16), 1,048,576 reports per launch) and, for k_hpke_open, "
             "bench.py --role hpke --reports 262144", ""]
    fetch, write, sq = {}, {}, {}
    for pre in ("", "hpke_"):
        stats = os.path.join(src, pre + "trace", "run_kernel_stats.csv")
        if not os.path.exists(stats):
            continue
        lines.append(f"## --kernel-trace --stats (per kernel){' -- bench.py --role hpke' if pre else ''}")
        lines.append(f"{'kernel':40s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} {'pct':>7s}")
        with open(stats) as f:
            for row in csv.DictReader(f):
                if row["Name"].startswith(("void at::", "at::", "__amd")):
                    continue
                lines.append(f"{short(row['Name']):40s} {row['Calls']:>6s} "
                             f"{float(row['AverageNs']) / 1e3:10.1f} {float(row['MinNs']) / 1e3:10.1f} "
                             f"{float(row['MaxNs']) / 1e3:10.1f} {float(row['Percentage']):7.2f}")
        lines.append("")
        for dst, name in ((fetch, "pmc_fetch"), (write, "pmc_write"), (sq, "pmc_sq"),
                          (sq, "pmc_stall")):
            for k, v in counters(os.path.join(src, pre + name, "run_counter_collection.csv")).items():
                if k.startswith("k_hpke") != bool(pre):
                    continue
                for c, vals in v.items():
                    dst.setdefault(k, {}).setdefault(c, vals)
    traffic = {}
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import isa_mix
    asm = {}
    for source in ("prio3_engine.hip", "hpke.hip"):
        asm.update(isa_mix.split_kernels(open(isa_mix.asm_path(source)).read().splitlines()))
    ceilings = {}
    for k, body in asm.items():
        loops = isa_mix.loops(body)
        lp = [isa_mix.mix(b) for _, b in loops]
        lp = [c for c in lp if c["full"] + c["half"] >= 50]
        c = max(lp, key=lambda c: c["full"] + c["half"]) if lp else isa_mix.mix(body)
        if isa_mix.demangle(k) == "k_hpke_open":
            # the Montgomery-ladder loop (most v_mad_u64_u32; 255 iterations per report, ~90 %
            # of the dynamic instructions) rather than the largest static loop (GHASH/AES)
            lb = max((b for _, b in loops),
                     key=lambda b: sum(1 for ln in b if ln.strip().startswith("v_mad_u64_u32")))
            c = isa_mix.mix(lb)
        base = isa_mix.demangle(k)
        if base not in ceilings:  # first instantiation in the file: the Fp128 / <2,32> one
            ceilings[base] = dict(valu_ceiling_T=isa_mix.ceiling(c),
                                  half_frac=c["half"] / max(1, c["full"] + c["half"]))
    lines += ["", "## HBM traffic per launch (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; KiB -> bytes)",
              f"{'kernel':40s} {'fetch_MB':>10s} {'write_MB':>10s} {'total_MB':>10s}"]
    for k in sorted(set(fetch) | set(write)):
        if k.startswith(("at::", "__amd", "vectorized", "elementwise", "reduce_kernel")):
            continue
        fv, wv = fetch.get(k, {}).get("FETCH_SIZE", []), write.get(k, {}).get("WRITE_SIZE", [])
        if not fv or not wv:
            continue
        fb = 2 * 1024 * sum(fv) / len(fv)
        wb = 1024 * sum(wv) / len(wv)
        traffic[k] = dict(fetch_bytes=fb, write_bytes=wb, bytes=fb + wb)
        lines.append(f"{k:40s} {fb / 1e6:10.1f} {wb / 1e6:10.1f} {(fb + wb) / 1e6:10.1f}")
    lines += ["", "## SQ / GRBM counters per launch"]
    names = sorted({c for k in sq for c in sq[k]})
    for k in sorted(sq):
        if k.startswith(("at::", "__amd", "vectorized", "elementwise", "reduce_kernel")):
            continue
        lines.append(k)
        for c in names:
            if sq[k].get(c):
                lines.append(f"    {c:24s} {sum(sq[k][c]) / len(sq[k][c]):20.0f}")
    txt = "\n".join(lines) + "\n"
    with open(os.path.join(ROOT, "profiles", f"{tag}_rocprof_summary.txt"), "w") as f:
        f.write(txt)
    kernels = {}
    for k, v in traffic.items():
        base = re.sub(r"<.*", "", k)
        d = dict(v)
        if k in sq and sq[k].get("SQ_WAVES"):
            d["valu_instr_per_item"] = (sum(sq[k]["SQ_INSTS_VALU"]) / len(sq[k]["SQ_INSTS_VALU"]) /
                                        (sum(sq[k]["SQ_WAVES"]) / len(sq[k]["SQ_WAVES"])))
        d.update(ceilings.get(base, {}))
        kernels[base] = d
    # WRITE_SIZE counts L2 lines when they reach memory: the dirty lines k_prep_h leaves in L2
    # are written back while the next kernel of the step runs (k_slow_redo, which returns at once
    # when no report is flagged), so those bytes are k_prep_h's
    if "k_prep_h" in kernels and "k_slow_redo" in kernels:
        wb = kernels["k_slow_redo"]["write_bytes"]
        kernels["k_prep_h"]["writeback_after_kernel_bytes"] = wb
        kernels["k_prep_h"]["write_bytes"] += wb
        kernels["k_prep_h"]["bytes"] += wb
        kernels["k_slow_redo"]["write_bytes"] = 0.0
        kernels["k_slow_redo"]["bytes"] = kernels["k_slow_redo"]["fetch_bytes"]
        txt += (f"\n# k_slow_redo's WRITE_SIZE ({wb / 1e6:.1f} MB) is k_prep_h's L2 write-back, "
                "attributed to k_prep_h in kernel_counts.json\n")
        with open(os.path.join(ROOT, "profiles", f"{tag}_rocprof_summary.txt"), "w") as f:
            f.write(txt)
    # kernels this pass did not run (e.g. SKIP_HPKE) keep their earlier entry and its source
    path = os.path.join(ROOT, "profiles", "kernel_counts.json")
    src = f"profiles/{tag}_rocprof_summary.txt"
    merged = {}
    if os.path.exists(path):
        with open(path) as f:
            old = json.load(f)
        for k, v in old.get("kernels", {}).items():
            if k not in kernels:
                merged[k] = dict(v, source=v.get("source", old.get("source")))
    for k, v in kernels.items():
        merged[k] = dict(v, source=src)
    with open(path, "w") as f:
        json.dump(dict(tag=tag, source=src, kernels=merged), f, indent=1)
    print(txt)


if __name__ == "__main__":
    main()
