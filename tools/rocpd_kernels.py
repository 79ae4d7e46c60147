"""Per-kernel stats from a rocprofv3 rocpd database (ROCm 7.2 writes SQLite by default):
usage: rocpd_kernels.py <run_results.db> <out.csv>.  Columns: kernel, calls, total_ms,
avg_ms, min_ms, max_ms, grid_x of the largest dispatch, and the calls / average over the
dispatches of that largest grid (the whole-shard decode of bench.py; smaller dispatches are the
header probe, the guess cache and the parity splits)."""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = {}
    durs = {}
    for name, dur, gx in c.execute("select name, duration, grid_x from kernels"):
        durs.setdefault(name.split("(")[0], []).append((gx, dur / 1e6))
        short = name.split("(")[0]
        r = rows.setdefault(short, [0, 0.0, 1e30, 0.0, 0])
        r[0] += 1
        r[1] += dur / 1e6
        r[2] = min(r[2], dur / 1e6)
        r[3] = max(r[3], dur / 1e6)
        r[4] = max(r[4], gx)
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ms", "avg_ms", "min_ms", "max_ms", "max_grid_x",
                    "calls_max_grid", "avg_ms_max_grid"])
        for k, r in sorted(rows.items(), key=lambda kv: -kv[1][1]):
            big = [d for g, d in durs[k] if g == r[4]]
            w.writerow([k, r[0], round(r[1], 3), round(r[1] / r[0], 3), round(r[2], 3),
                        round(r[3], 3), r[4], len(big), round(sum(big) / len(big), 3)])
    print(open(out).read())


if __name__ == "__main__":
    main()
