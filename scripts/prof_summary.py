"""Kernel-time summary of a rocprofv3 run database (rocpd sqlite): per kernel name, calls,
total / mean / max duration (ms), share of GPU time.  Usage: prof_summary.py <run_results.db>
[name-filter]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = {}
    for name, s, e in rows:
        if filt and filt not in name:
            continue
        d = (e - s) / 1e6
        a = agg.setdefault(name, [0, 0.0, 0.0])
        a[0] += 1
        a[1] += d
        a[2] = max(a[2], d)
    tot = sum(a[1] for a in agg.values()) or 1.0
    print(f"{'kernel':70s} {'calls':>7s} {'total_ms':>10s} {'mean_ms':>9s} {'max_ms':>9s} {'pct':>6s}")
    for name, (n, t, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{name[:70]:70s} {n:7d} {t:10.3f} {t / n:9.4f} {mx:9.4f} {100 * t / tot:6.2f}")


if __name__ == "__main__":
    main()
