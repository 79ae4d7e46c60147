"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, restricted to each kernel's
largest-grid dispatches (the whole-shard decode of bench.py; the smaller dispatches are the
header probe, the guess cache and the parity splits).  usage:
trace_kernels.py <run_kernel_trace.csv> <out.csv> [kernel-substring ...]"""
import csv
import sys


def main():
    src, out = sys.argv[1], sys.argv[2]
    want = sys.argv[3:]
    rows = {}
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"].split("(")[0]
        if want and not any(w in name for w in want):
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        rows.setdefault(name, []).append((grid, dur))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid", "calls_at_grid", "avg_ms", "min_ms", "max_ms", "all_calls"])
        for name, v in sorted(rows.items(), key=lambda kv: -max(d for _, d in kv[1])):
            g = max(x for x, _ in v)
            d = [t for x, t in v if x == g]
            w.writerow([name, g, len(d), round(sum(d) / len(d), 4), round(min(d), 4), round(max(d), 4), len(v)])
    print(open(out).read())


if __name__ == "__main__":
    main()
