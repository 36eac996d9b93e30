"""Summarise a rocprofv3 kernel trace (SQLite .db or kernel_stats/kernel_trace CSV):
per-kernel total/avg time and share of GPU time; optionally only the last K steps."""
import csv
import glob
import os
import sqlite3
import sys


def load(path):
    rows = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, dur, grid in c.execute("select name, duration, grid_x from kernels order by start"):
            rows.append((name, dur, grid))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r.get("Grid_Size_X")))
    return rows


def short(n):
    for p in ("void ", "(anonymous namespace)::", "_ZN12_GLOBAL__N_1"):
        n = n.replace(p, "")
    n = n.split("(")[0]
    return n[:70]


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) + \
            glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        path = cands[0]
    rows = load(path)
    agg = {}
    for name, dur, _ in rows:
        k = short(name)
        t, c = agg.get(k, (0, 0))
        agg[k] = (t + dur, c + 1)
    total = sum(t for t, _ in agg.values())
    print(f"source: {path}\ntotal kernel time {total / 1e6:.3f} ms over {len(rows)} dispatches")
    print(f"{'kernel':72s} {'calls':>6s} {'total ms':>10s} {'avg us':>9s} {'%':>6s}")
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:40]:
        print(f"{k:72s} {c:6d} {t / 1e6:10.3f} {t / c / 1e3:9.1f} {100 * t / total:6.2f}")


if __name__ == "__main__":
    main()
