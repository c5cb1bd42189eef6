"""Per-kernel statistics from a rocprofv3 rocpd database (run_results.db): calls, total, average,
min and max duration, and the gaps between consecutive dispatches on the GPU, for profiles/."""
import sqlite3
import sys
from collections import defaultdict


def stats(db, top=25):
    con = sqlite3.connect(db)
    cur = con.cursor()
    cols = [c[1] for c in cur.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = cur.execute(f"select {name}, start, end from kernels order by start").fetchall()
    agg = defaultdict(list)
    for n, s, e in rows:
        short = n.split("(")[0].replace("void ", "")
        agg[short].append((e - s) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    out = [f"{'kernel':60s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}"]
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
        out.append(f"{k[:60]:60s} {len(v):7d} {sum(v) / 1e3:10.3f} {sum(v) / len(v):9.1f} "
                   f"{min(v):9.1f} {max(v):9.1f} {100 * sum(v) / tot:6.1f}")
    if rows:
        span = (rows[-1][2] - rows[0][1]) / 1e6
        out.append(f"span {span:.3f} ms, busy {tot / 1e3:.3f} ms ({100 * tot / 1e3 / span:.1f} %), "
                   f"{len(rows)} dispatches")
    return "\n".join(out)


if __name__ == "__main__":
    for db in sys.argv[1:]:
        print(db)
        print(stats(db))
