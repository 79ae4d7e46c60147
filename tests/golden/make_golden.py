"""Regenerates the committed golden fixtures (tests/golden/).

Inputs: small_pe.bam (config #1 stand-in: the reference ships no BAM fixture)
and edge-case BAMs, all from tools/gen_bam.cpp with fixed seeds.  Expected outputs: the CPU
oracle's split read, split list and guesses (oracle/hbam_oracle.c), plus zlib/libdeflate
inflate digests.  Run:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")]
import genbam  # noqa: E402
import oracle  # noqa: E402
from conftest import SMALL_PE_PARAMS  # noqa: E402

EDGE = {
    # htslib packing (records never straddle), empty blocks mid-file, ragged records
    "edge_htslib_empty.bam": dict(records=6000, seed=11, straddle=0, empty_every=7, odd_every=13),
    # uniform qualities (poor compression), records > 64 KiB spanning blocks
    "edge_uniform_long.bam": dict(records=4000, seed=12, uniform_qual=1, long_every=500),
    # unsorted, no terminator, level 1
    "edge_unsorted_l1.bam": dict(records=5000, seed=13, sorted=0, level=1, terminator=0),
}


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def expected(data):
    h = oracle.read_header(data)
    r = oracle.read_split(data, h["first_voffset"], (len(data) << 16) | 0xffff)
    out = dict(header=h, n=r["n"], status=r["status"], err_record=r["err_record"],
               var_sha=digest(r["var"]))
    for k, _ in oracle.FIXED_FIELDS:
        out[k + "_sha"] = digest(r[k])
    blocks = oracle.scan_blocks(data)
    u = b"".join(zlib.decompressobj(-15).decompress(bytes(data[int(c) + 18:int(c) + int(l) - 8]))
                 for c, l in zip(blocks["coff"], blocks["clen"]))
    out["n_blocks"] = len(blocks["coff"])
    out["inflated_sha"] = hashlib.sha256(u).hexdigest()
    out["inflated_len"] = len(u)
    # probabilistic splits at three split sizes + guesses at fixed offsets
    out["splits"] = {}
    for ss in (64 << 10, 256 << 10, 1 << 20):
        b, e = oracle.file_splits(len(data), ss)
        res = oracle.probabilistic_splits(data, b, e)
        out["splits"][str(ss)] = (res if isinstance(res, int) else
                                 [[int(x), int(y)] for x, y in zip(*res)])
    rng = np.random.default_rng(3)
    begs = sorted(int(x) for x in rng.integers(0, len(data), 64))
    out["guesses"] = [[b, *oracle.guess_bam_record_start(data, b, len(data), h["n_ref"])]
                      for b in begs]
    return out


def main():
    files = {"small_pe.bam": SMALL_PE_PARAMS, **EDGE}
    table = {}
    for name, kw in files.items():
        data = np.asarray(genbam.generate(**kw))
        data.tofile(os.path.join(HERE, name))
        table[name] = dict(params=kw, expected=expected(data))
        print(name, len(data), table[name]["expected"]["n"])
    with open(os.path.join(HERE, "expected.json"), "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
