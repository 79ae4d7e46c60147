"""Fold the two rocprofv3 passes of tools/pmc_calib (FETCH_SIZE, WRITE_SIZE) into per-shape
calibration factors: counted bytes (KiB -> B) / known bytes of each kernel.

usage: pmc_calib.py <calib_stdout.txt> <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>
"""
import csv
import json
import sys


def counters(path, name):
    out = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != name:
            continue
        k = row["Kernel_Name"].split("(")[0].strip()
        out.setdefault(k, []).append(float(row["Counter_Value"]) * 1024.0)
    return out


def main():
    log, fcsv, wcsv, out = sys.argv[1:5]
    known = {}
    for ln in open(log):
        if ln.startswith("k_"):
            f = ln.split(None, 2)
            known[f[0]] = (int(f[1]), f[2].strip())
    fe = counters(fcsv, "FETCH_SIZE")
    wr = counters(wcsv, "WRITE_SIZE")
    res = {}
    for k, (b, what) in known.items():
        fb = max(fe.get(k, [0.0]))
        wb = max(wr.get(k, [0.0]))
        res[k] = {"known_bytes": b, "what": what, "fetch_counted": fb, "write_counted": wb,
                  "fetch_over_known": round(fb / b, 4), "write_over_known": round(wb / b, 4)}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        print("%-20s known %14d  FETCH/known %.3f  WRITE/known %.3f  %s" % (
            k, v["known_bytes"], v["fetch_over_known"], v["write_over_known"], v["what"]))


if __name__ == "__main__":
    main()
