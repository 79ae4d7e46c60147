"""Whole-block dataflow depth of the LZ77 pass (tooling; the round-5 verdict's "one BGZF block per
workgroup, history in LDS" option): every match of a block is cut into <= 16-byte units as
k_resolve_units cuts them (resolve_units.h; short periods read the bytes before the match), and
each unit's round is 1 + the latest round of the bytes its source reads (literals: round 0).  The
depth is the number of dataflow rounds a block needs when its whole history is resident; units
per round is the parallelism one block offers.

    python tools/lz77_depth_sim.py FILE.bam [--blocks N] [--skip K]
"""
import argparse
import collections
import os
import statistics
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from deflate_trace import trace  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("bam")
    ap.add_argument("--blocks", type=int, default=120)
    ap.add_argument("--skip", type=int, default=2, help="leading blocks to skip (header)")
    a = ap.parse_args()
    data = open(a.bam, "rb").read(80 << 20)
    o = nb = units_tot = 0
    depths = []
    hist = collections.Counter()
    while o + 18 <= len(data) and len(depths) < a.blocks:
        bsize = struct.unpack_from("<H", data, o + 16)[0] + 1
        raw = data[o + 18:o + bsize - 8]
        o += bsize
        nb += 1
        if nb <= a.skip:
            continue
        _, toks, out = trace(raw)
        rnd = bytearray(out)
        maxr = 0
        for t in toks:
            if t[2] != "match":
                continue
            p, (ln, d) = t[1], t[3]
            for q in range(p, p + ln, 16):
                n = min(16, p + ln - q)
                s0, s1 = (q - d, q - d + n) if (d >= 16 or d >= ln) else (p - d, p)
                r = 1 + max(rnd[s0:s1])
                rnd[q:q + n] = bytes([min(r, 255)]) * n
                hist[r] += 1
                units_tot += 1
                maxr = max(maxr, r)
        depths.append(maxr)
    print("blocks %d: depth mean %.1f min %d max %d; units per block %.0f; units per round %.1f"
          % (len(depths), statistics.mean(depths), min(depths), max(depths), units_tot / len(depths),
             units_tot / sum(depths)))
    cum = 0
    for r in sorted(hist):
        cum += hist[r]
        if r <= 8 or r % 20 == 0:
            print("  round %3d: %6d units, cumulative %.3f" % (r, hist[r], cum / units_tot))


if __name__ == "__main__":
    main()
