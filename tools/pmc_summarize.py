"""Fold two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs) over one decode into
per-kernel HBM traffic, and the Huffman pass's entry that bench.py reads as roofline.traffic.

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section, checked on this repository's
own access shapes by tools/pmc_calib.hip -> profiles/r04/calib/):
  * FETCH_SIZE and WRITE_SIZE are reported in KiB;
  * FETCH_SIZE counts 64 B per 128-B L2->fabric request, so it is doubled.  The guide states this
    for 16-B-per-lane streaming reads; the calibration finds the same factor for every read shape
    of the pipeline once bytes are counted as 128-B lines touched: streaming 16 B/lane 0.500
    (model 0.5), 16-B units at +3 0.516, random 8-byte loads 8.41 per 8 B (model 16.96 / 2 = 8.48),
    36-B fixed parts at stride 340 2.30 (model 4.53 / 2 = 2.27);
  * WRITE_SIZE reads the bytes exactly (1.000 streaming, 1.152 for lane-per-64-KiB-region
    16-byte stores: partial lines at region edges);
  * FETCH counts L2 misses served by the 256 MiB Infinity Cache as well as HBM reads (guide,
    HBM section).  When a kernel's corrected bytes over its time exceed the achievable 6.3 TB/s,
    at least the excess came from the Infinity Cache: `hbm_bytes_max` caps the HBM share at
    6.3 TB/s x time and `mall_bytes_min` is the rest.

usage: pmc_summarize.py FETCH_CSV WRITE_CSV COMP_BYTES OUT_DIR TREE [STAGES_JSON]
  STAGES_JSON: a bench.py line (its stages_ms give each kernel's unprofiled time)
writes OUT_DIR/pmc_kernels.json (every kernel) and OUT_DIR/pmc_huffman.json (bench.py: the Huffman
pass, k_inflate_wave plus the lane-per-block k_inflate_tokens for the blocks it leaves)
"""
import csv
import json
import os
import sys

HBM_ACHIEVABLE = 6.3e12
STAGE_OF = {"k_inflate_wave": "huffman_ms", "k_inflate_tokens": "huffman_ms", "k_resolve": "resolve_ms", "k_resolve_units": "resolve_ms", "k_decode_pools": "pools_ms",
            "k_decode_fixed": "decode_ms", "k_scan_chunks": "scan_ms"}


def per_kernel(path, counter):
    """kernel -> list of per-dispatch values (KiB), summed over the counter's instances"""
    vals = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        k = row["Kernel_Name"].split("(")[0].strip()
        k = k[5:] if k.startswith("void ") else k
        k = k[6:] if k.startswith("hbam::") else k
        d = vals.setdefault(k, {})
        d[row["Dispatch_Id"]] = d.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return {k: list(v.values()) for k, v in vals.items()}


def main():
    fcsv, wcsv, comp, outdir, tree = sys.argv[1:6]
    stages = {}
    if len(sys.argv) > 6:
        stages = json.load(open(sys.argv[6])).get("stages_ms", {})
    f = per_kernel(fcsv, "FETCH_SIZE")
    w = per_kernel(wcsv, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        # the decode of the whole file is the largest dispatch (smaller ones: header probe)
        fetch = 2.0 * 1024.0 * max(f.get(k, [0.0]))
        write = 1024.0 * max(w.get(k, [0.0]))
        e = {"fetch_raw_kib": max(f.get(k, [0.0])), "write_raw_kib": max(w.get(k, [0.0])),
             "fetch_bytes": fetch, "write_bytes": write, "hbm_bytes_per_launch": fetch + write}
        ms = stages.get(STAGE_OF.get(k, ""), 0.0)
        if ms:
            t = ms / 1e3
            e["ms"] = ms
            e["implied_tb_s"] = round((fetch + write) / t / 1e12, 3)
            cap = HBM_ACHIEVABLE * t
            e["hbm_bytes_max"] = min(fetch + write, cap)
            e["mall_bytes_min"] = max(0.0, fetch + write - cap)
        res[k] = e
    os.makedirs(outdir, exist_ok=True)
    note = ("FETCH_SIZE x2 (128-B requests tallied at 64 B; calibrated per access shape: "
            "profiles/r04/calib/), KiB -> B; FETCH includes Infinity Cache hits")
    json.dump({"tree": tree, "comp_bytes": int(comp), "note": note, "kernels": res},
              open(os.path.join(outdir, "pmc_kernels.json"), "w"), indent=1)
    h = res.get("k_inflate_tokens")
    hw = res.get("k_inflate_wave")
    if hw and h and hw["hbm_bytes_per_launch"] < 0.01 * h["hbm_bytes_per_launch"]:
        del res["k_inflate_wave"]  # only a small call (the header probe) took the wave pass
    if h and "k_inflate_wave" not in res:  # a call above HBAM_WAVE_MAX_BLOCKS: the lane pass alone
        one = {"kernel": "k_inflate_tokens", "tree": tree, "comp_bytes": int(comp),
               "fetch_bytes_per_launch": h["fetch_bytes"], "write_bytes_per_launch": h["write_bytes"],
               "hbm_bytes_per_launch": h["hbm_bytes_per_launch"], "note": note}
        json.dump(one, open(os.path.join(outdir, "pmc_k_inflate_tokens.json"), "w"), indent=1)
    h = res.get("k_inflate_wave")
    if h:
        lane = res.get("k_inflate_tokens", {"fetch_bytes": 0.0, "write_bytes": 0.0})
        fb, wb = h["fetch_bytes"] + lane["fetch_bytes"], h["write_bytes"] + lane["write_bytes"]
        one = {"kernel": "k_inflate_wave", "tree": tree, "comp_bytes": int(comp),
               "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb, "hbm_bytes_per_launch": fb + wb,
               "note": note + "; k_inflate_wave + the k_inflate_tokens launch over the blocks it leaves"}
        json.dump(one, open(os.path.join(outdir, "pmc_huffman.json"), "w"), indent=1)
    for k, e in res.items():
        print("%-24s fetch %8.2f GB write %8.2f GB%s" % (k, e["fetch_bytes"] / 1e9, e["write_bytes"] / 1e9,
              ("  %.2f TB/s implied" % e["implied_tb_s"]) if "implied_tb_s" in e else ""))


if __name__ == "__main__":
    main()
