"""Summaries from a rocprofv3 SQLite (rocpd) output: per-kernel stats, and the kernel
timeline of the last N calls of a loop (gaps = host/launch overhead).

    python scripts/rocpd_summary.py gpurun_out/prof/run_results.db [--timeline 40]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--timeline", type=int, default=0)
    ap.add_argument("--csv", default=None, help="write the per-kernel stats here")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    rows = list(db.execute(f"select {name_col}, start, end from kernels order by start"))
    stats = {}
    for n, s, e in rows:
        d = stats.setdefault(n, [0, 0.0, float("inf"), 0.0])
        dt = (e - s) / 1e3
        d[0] += 1
        d[1] += dt
        d[2] = min(d[2], dt)
        d[3] = max(d[3], dt)
    tot = sum(v[1] for v in stats.values())
    out = ["Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs,Percentage"]
    for n, (c, t, mn, mx) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        out.append(f'"{n}",{c},{t * 1e3:.0f},{t / c * 1e3:.0f},{mn * 1e3:.0f},{mx * 1e3:.0f},{100 * t / tot:.2f}')
        print(f"{c:6d} {t / c:10.2f} us avg  {100 * t / tot:6.2f}%  {n[:110]}")
    if a.csv:
        open(a.csv, "w").write("\n".join(out) + "\n")
    if a.timeline:
        tl = rows[-a.timeline:]
        t0 = tl[0][1]
        prev = t0
        for n, s, e in tl:
            print(f"{(s - t0) / 1e3:10.1f} us  gap {(s - prev) / 1e3:8.1f}  dur {(e - s) / 1e3:8.1f}  {n[:80]}")
            prev = e


if __name__ == "__main__":
    main()
