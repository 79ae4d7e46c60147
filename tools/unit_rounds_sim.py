"""Dependency rounds of k_resolve_units' ordered units (resolve_units.h) on real DEFLATE blocks, on
the CPU, for two ways of cutting a short-period match (distance < 16 < length) into units:

  chain   (the shipped rule)  a head unit from the period, then units at distance
          dist * ceil(16 / dist) (dist < 8) or 2 * dist (8 <= dist < 16): every unit of the match
          reads the one before it, so a 258-byte run of one byte is 17 rounds deep;
  period  every unit reads the dist bytes before the match and rotates them by its offset, so
          all units of the match depend only on bytes before it.

Per 1 KiB stretch: units whose source ends before the stretch are "pre" (copied before the
rounds); a round copies every ordered unit with no pending byte in its source.

    python tools/unit_rounds_sim.py [--size BYTES] [--blocks N]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from deflate_trace import bgzf_payload, trace  # noqa: E402

S = 1024


def units_of(p, ln, d, rule):
    """(dest start, bytes, source start, source end) per unit of match (p, ln, d)"""
    out = []
    if d >= ln or d >= 16:
        for q in range(p, p + ln, 16):
            n = min(16, p + ln - q)
            out.append((q, n, q - d, q - d + n))
        return out
    if rule == "period":
        for q in range(p, p + ln, 16):
            out.append((q, min(16, p + ln - q), p - d, p))
        return out
    if d < 8:
        h = min(16, ln)
        D = d * -(-16 // d)
    else:
        h = d
        D = 2 * d
    out.append((p, h, p - d, p))
    for q in range(p + h, p + ln, 16):
        n = min(16, p + ln - q)
        out.append((q, n, q - D, q - D + n))
    return out


def stretch_rounds(raw, rule):
    _, toks, out = trace(raw)
    M = [(t[1], t[3][0], t[3][1]) for t in toks if t[2] == "match"]
    res = []
    for k in range((out + S - 1) // S):
        s0 = k * S
        us = [u for p, ln, d in M if s0 <= p < s0 + S for u in units_of(p, ln, d, rule)]
        pre = [u for u in us if u[3] <= s0]
        live = [u for u in us if u[3] > s0]
        nord = len(live)
        pend = set()
        for q, n, _, _ in live:
            pend.update(range(q, q + n))
        per = []
        while live:
            ready = [u for u in live if not any(x in pend for x in range(max(u[2], s0), u[3]))]
            if not ready:
                raise RuntimeError("no progress")
            for q, n, _, _ in ready:
                pend.difference_update(range(q, q + n))
            live = [u for u in live if u not in ready]
            per.append(len(ready))
        res.append((len(pre), nord, per))
    return res


def members(data):
    off = 0
    while off + 18 <= len(data):
        bsize = (data[off + 16] | data[off + 17] << 8) + 1
        yield data[off:off + bsize]
        off += bsize


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=float, default=4e6)
    ap.add_argument("--blocks", type=int, default=12)
    ap.add_argument("--seed", type=int, default=2)
    a = ap.parse_args()
    import numpy as np
    import genbam
    data = bytes(np.asarray(genbam.generate(target_bytes=int(a.size), seed=a.seed)))
    ms = [m for m in members(data) if len(m) > 1000]
    step = max(1, len(ms) // a.blocks)
    pick = ms[1::step][:a.blocks]
    for rule in ("chain", "period"):
        st = []
        for m in pick:
            st += stretch_rounds(bgzf_payload(m), rule)
        n = len(st)
        rounds = sum(len(p) for _, _, p in st)
        print("%-6s stretches %d: pre units %.1f, ordered units %.1f, rounds %.2f per stretch; "
              "rounds per stretch histogram %s" % (
                  rule, n, sum(s[0] for s in st) / n, sum(s[1] for s in st) / n, rounds / n,
                  dict(sorted(collections.Counter(len(p) for _, _, p in st).items()))), flush=True)


if __name__ == "__main__":
    main()
