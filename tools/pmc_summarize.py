"""Fold rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE) for one kernel into
profiles/pmc_inflate.json, which bench.py reads as roofline.traffic.

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE
are reported in KiB; on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane reads, so it
is doubled.  usage: pmc_summarize.py <fetch_csv> <write_csv> <kernel-substring> <comp_bytes> <out> [tree]
"""
import csv
import json
import sys


def per_dispatch(path, kernel, counter):
    vals = {}
    for row in csv.DictReader(open(path)):
        if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
            vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fcsv, wcsv, kern, comp, out = sys.argv[1:6]
    tree = sys.argv[6] if len(sys.argv) > 6 else "round3"
    f = per_dispatch(fcsv, kern, "FETCH_SIZE")
    w = per_dispatch(wcsv, kern, "WRITE_SIZE")
    assert f and w, "no dispatches of %s" % kern
    # the decode of the whole file is the largest dispatch (smaller ones: header probe)
    fetch = 2.0 * 1024.0 * max(f)
    write = 1024.0 * max(w)
    res = {"kernel": kern, "tree": tree, "comp_bytes": int(comp), "dispatches": [len(f), len(w)],
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": fetch + write,
           "note": "FETCH_SIZE x2 (gfx950 16-B/lane read correction), KiB -> B"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
