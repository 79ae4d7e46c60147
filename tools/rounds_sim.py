"""LZ77-pass dependency model (k_resolve, resolve_dev.h) on real DEFLATE blocks, on the CPU:
per 1 KiB stretch, the "ordered" matches (external source ending inside the stretch) and how
many of them each dataflow round of the r02 pass resolves (round 1 = sources with no pending
byte).  Used to size the round-1 + in-order tail scheme (HBAM_RS_SERIAL).

    python tools/rounds_sim.py BLOCK.bgzf [...]
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from deflate_trace import bgzf_payload, trace  # noqa: E402

S = 1024


def stretch_rounds(raw):
    blocks, toks, out = trace(raw)
    M = [(t[1], t[3][0], t[3][1]) for t in toks if t[2] == "match"]
    res = []
    for k in range((out + S - 1) // S):
        s0 = k * S
        ordered = [(p, l, d, p - d + min(l, d)) for p, l, d in M if s0 <= p < s0 + S and p - d + min(l, d) > s0]
        pend = set()
        for p, l, d, e in ordered:
            pend.update(range(p, p + l))
        live, per = list(ordered), []
        while live:
            ready = [m for m in live if not any(x in pend for x in range(max(m[0] - m[2], s0), m[3]))]
            for m in ready:
                pend.difference_update(range(m[0], m[0] + m[1]))
            live = [m for m in live if m not in ready]
            per.append(len(ready))
        res.append((len(ordered), per))
    return len(M), res


def main():
    for path in sys.argv[1:]:
        nm, st = stretch_rounds(bgzf_payload(open(path, "rb").read()))
        tot = sum(n for n, _ in st)
        r1 = sum(p[0] for n, p in st if p)
        print("%s: matches %d, ordered %d, rounds %d, round 1 %d, after round 1 %d (%.1f per stretch); "
              "rounds per stretch %s" % (path, nm, tot, sum(len(p) for _, p in st), r1, tot - r1,
                                          (tot - r1) / max(1, len(st)),
                                          dict(sorted(collections.Counter(len(p) for _, p in st).items()))))


if __name__ == "__main__":
    main()
