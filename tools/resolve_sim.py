"""CPU replay of k_resolve's stretch schedule over real DEFLATE blocks (the blocks file of
tools/cpu_model/make_blocks.py): per 1 KiB stretch, the matches whose source is older than the
LDS window ("far": read from ubuf), the distinct 128-B lines those reads touch, how far back they
reach, and the number of ordered matches per stretch with the width of their dependency ranges
(k_resolve this round).

    python tools/resolve_sim.py BLOCKS.bin [--every 12] [--window 512]
"""
import argparse
import collections
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from deflate_trace import trace  # noqa: E402

S = 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("blocks")
    ap.add_argument("--every", type=int, default=12, help="sample every k-th block")
    ap.add_argument("--window", type=int, default=512)
    a = ap.parse_args()
    f = open(a.blocks, "rb")
    magic, n = struct.unpack("<II", f.read(8))
    back = collections.Counter()
    nord_h = collections.Counter()
    dep_w = collections.Counter()
    nblk = nm = nfar = lines = nst = 0
    for b in range(n):
        clen, isz = struct.unpack("<II", f.read(8))
        raw = f.read(clen)
        f.read(isz)
        if b % a.every:
            continue
        _, toks, out = trace(raw)
        nblk += 1
        M = [(t[1], t[3][0], t[3][1]) for t in toks if t[2] == "match"]
        per = collections.defaultdict(set)
        for p, ln, d in M:
            nm += 1
            s0 = (p // S) * S
            src = p - d
            if src + a.window < s0:
                nfar += 1
                back[min((s0 - src) // 1024, 32)] += 1
                for x in range(src // 128, (src + min(ln, d) - 1) // 128 + 1):
                    per[s0].add(x)
        lines += sum(len(v) for v in per.values())
        for k in range((out + S - 1) // S):
            s0 = k * S
            ordm = [(p, ln, d) for p, ln, d in M if s0 <= p < s0 + S and p - d + min(ln, d) > s0]
            nst += 1
            nord_h[min(len(ordm) // 16, 20)] += 1
            for i, (p, ln, d) in enumerate(ordm):
                lo, e = p - d, p - d + min(ln, d)
                deps = [j for j, (q, m, _) in enumerate(ordm[:i]) if q < e and q + m > lo]
                dep_w[min(deps[-1] - deps[0] + 1, 8) if deps else 0] += 1
    print("blocks %d  matches/block %.0f  far/block %.0f (%.1f %%)  far 128-B lines/block %.0f"
          % (nblk, nm / nblk, nfar / nblk, 100.0 * nfar / nm, lines / nblk))
    tot, c = sum(back.values()), 0
    for k in sorted(back):
        c += back[k]
        print("far source %2d KiB behind the stretch: %5.1f %%  cumulative %5.1f %%" % (k, 100.0 * back[k] / tot, 100.0 * c / tot))
    tot, c = sum(nord_h.values()), 0
    for k in sorted(nord_h):
        c += nord_h[k]
        print("ordered matches %3d-%3d per stretch: %5.1f %%  cumulative %5.1f %%" % (16 * k, 16 * k + 15, 100.0 * nord_h[k] / tot, 100.0 * c / tot))
    print("dependency range widths (0 = none):", sorted(dep_w.items()))


if __name__ == "__main__":
    main()
