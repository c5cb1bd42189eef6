"""Reads the jobs lines' evidence: rocprofv3 kernel traces (rocpd run_results.db)
and the executor's group trace (JANUS_EXEC_TRACE files) of `bench.py --role jobs` runs.

  python tools/jobs_trace.py db  <run_results.db> [KERNEL [LAST]]   per-kernel time over the timed
        region (the last LAST launches of KERNEL, default k_prep_h / 70), GPU busy fraction, the
        queues the groups ran on, and every stall (> 3 median periods) between consecutive groups
  python tools/jobs_trace.py exec <trace> [<trace> ...]              per run: mean group size, how
        long the launcher waited for a group's writers after taking it, staged -> done, and the
        period between consecutive groups (a group every N us)
"""
import json
import os
import sqlite3
import statistics as S
import sys
from collections import Counter, defaultdict


def _short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")


def db(path, key="k_prep_h", last=70):
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end, queue_id, stream_id from kernels "
                     "order by start").fetchall()
    rows = [(_short(r[0]),) + tuple(r[1:]) for r in rows]
    G = [r for r in rows if key in r[0]][-last:]
    if not G:
        return f"{path}: no {key} launches"
    t0, t1 = G[0][1], G[-1][2]
    W = [r for r in rows if r[1] >= t0 and r[2] <= t1]
    by = defaultdict(list)
    for r in W:
        by[r[0]].append((r[2] - r[1]) / 1e3)
    out = [f"{path}: timed region {(t1 - t0) / 1e6:.2f} ms, last {len(G)} {key} launches"]
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:10]:
        out.append(f"  {k[:40]:40s} n {len(v):4d} total {sum(v) / 1e3:7.2f} ms "
                   f"avg {S.mean(v):7.1f} us")
    iv = sorted((r[1], r[2]) for r in W)
    busy, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    out.append(f"  GPU busy {busy / 1e6:.2f} ms ({100 * busy / (t1 - t0):.0f} %); {key} queues "
               f"{dict(Counter(r[3] for r in G))}")
    per = [(G[i + 1][1] - G[i][1]) / 1e3 for i in range(len(G) - 1)]
    med = S.median(per)
    out.append(f"  {key} start to start: median {med:.0f} us, max {max(per):.0f} us")
    for i, g in enumerate(per):
        if g > 3 * med:  # a stall: more than three ordinary periods between two groups
            out.append(f"  gap {g:.0f} us between groups {i} and {i + 1}: queue {G[i][3]} -> "
                       f"{G[i + 1][3]}, stream {G[i][4]} -> {G[i + 1][4]}")
    return "\n".join(out)


def exec_trace(path, last=70):
    L = [list(map(float, ln.split())) for ln in open(path) if ln.strip()][-last:]
    js = path[:-len(".trace")] + ".json"
    v = json.load(open(js))["value"] / 1e6 if os.path.exists(js) else float("nan")
    ret = [t[3] for t in L]
    per = [ret[i + 1] - ret[i] for i in range(len(ret) - 1)]
    return (f"{os.path.basename(path)}: {v:.1f} M/s; group {S.mean(t[5] for t in L):.0f} reports; "
            f"writers after take {S.mean(t[2] - t[1] for t in L):.0f} us; staged -> done "
            f"{S.mean(t[3] - t[2] for t in L):.0f} us; a group every {S.mean(per):.0f} us "
            f"(max {max(per):.0f})")


if __name__ == "__main__":
    if sys.argv[1] == "db":
        print(db(sys.argv[2], *(sys.argv[3:4] or ["k_prep_h"]),
                 *([int(sys.argv[4])] if len(sys.argv) > 4 else [])))
    else:
        for p in sys.argv[2:]:
            print(exec_trace(p))
