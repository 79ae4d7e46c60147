"""Fold the SQ PMC pass of tools/pmc_sq.sh into per-kernel ratios (largest dispatch of each
kernel): issue/wait split of SQ_WAVE_CYCLES and the LDS bank-conflict share of LDS cycles.
usage: pmc_sq_summarize.py <run_counter_collection.csv> <out.json>"""
import collections
import csv
import json
import sys


def main():
    src, out = sys.argv[1:3]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(src)):
        k = r["Kernel_Name"].split("(")[0].replace("hbam::", "")
        agg[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[(k, r["Dispatch_Id"])] = dict(vgpr=int(r["VGPR_Count"]), lds=int(r["LDS_Block_Size"]),
                                           wg=int(r["Workgroup_Size"]), grid=int(r["Grid_Size"]))
    res = {}
    for (k, d), v in agg.items():
        if k in res and res[k]["counters"]["SQ_WAVE_CYCLES"] >= v["SQ_WAVE_CYCLES"]:
            continue
        wc = v["SQ_WAVE_CYCLES"]
        res[k] = {"dispatch": d, **meta[(k, d)], "counters": dict(v),
                  "active_inst_frac": v["SQ_ACTIVE_INST_ANY"] / wc,
                  "wait_any_frac": v["SQ_WAIT_ANY"] / wc,
                  "wait_inst_frac": v["SQ_WAIT_INST_ANY"] / wc,
                  "lds_conflict_frac_of_lds_cycles": v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_LDS_IDX_ACTIVE"], 1)}
    json.dump(res, open(out, "w"), indent=1)
    for k, r in res.items():
        print(k, {x: round(r[x], 3) for x in r if x.endswith("frac") or x.endswith("cycles")})


if __name__ == "__main__":
    main()
