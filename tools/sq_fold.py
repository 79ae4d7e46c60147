"""Fold several rocprofv3 --pmc SQ passes (one counter_collection.csv each, the same decode) into
per-kernel issue / wait splits: summed over every dispatch of a kernel, SQ_WAVE_CYCLES and the
SQ_WAIT_* / SQ_ACTIVE_* counters in quad-cycles, instruction counts per class.
usage: sq_fold.py OUT.json "what" pass1.csv [pass2.csv ...]"""
import collections
import csv
import json
import re
import sys


def kname(s):
    s = s.split("(")[0]
    s = re.sub(r"^void ", "", s).replace("hbam::", "")
    return re.sub(r"<.*>", "", s)


def main():
    out, what, srcs = sys.argv[1], sys.argv[2], sys.argv[3:]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for src in srcs:
        for r in csv.DictReader(open(src)):
            k = kname(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    res = {"what": what, "kernels": {}}
    for k, v in sorted(agg.items()):
        wc = v.get("SQ_WAVE_CYCLES", 0.0)
        if wc <= 0 or not k.startswith("k_"):
            continue
        e = {"dispatches": len(disp[k]), "counters": dict(v)}
        for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if c in v:
                e[c.lower().replace("sq_", "") + "_frac"] = round(v[c] / wc, 4)
        if v.get("SQ_WAVES"):
            e["insts_valu_per_wave"] = round(v.get("SQ_INSTS_VALU", 0) / v["SQ_WAVES"], 1)
            e["insts_salu_per_wave"] = round(v.get("SQ_INSTS_SALU", 0) / v["SQ_WAVES"], 1)
            e["wave_quad_cycles_per_wave"] = round(wc / v["SQ_WAVES"], 1)
        if v.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_conflict_frac"] = round(v.get("SQ_LDS_BANK_CONFLICT", 0) / v["SQ_LDS_IDX_ACTIVE"], 4)
        res["kernels"][k] = e
        print(k, {x: y for x, y in e.items() if x != "counters"})
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
