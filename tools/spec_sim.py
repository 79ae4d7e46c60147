"""Sizing study for a wave-per-block Huffman pass that decodes one BGZF block with 64 lanes
from speculative bit offsets (DESIGN.md §7, round 4 close): per BGZF block of the bench's
generator (tools/genbam, zlib level 5), the DEFLATE blocks and their symbol counts, and for
random start bits inside a block's symbol region how many tokens a decoder started there runs
before it lands on a true token boundary (then it is in step with the true decode for good).

    python tools/spec_sim.py [MB] [--starts 64]
"""
import argparse
import os
import random
import struct
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import genbam  # noqa: E402
from deflate_trace import Bits, LBASE, LEXT, DBASE, DEXT, canon, trace  # noqa: E402


def lut(table):
    """(code, length) -> symbol  as a 15-bit LSB-first lookup: v & ((1<<L)-1) -> (sym, L)"""
    t = [None] * (1 << 15)
    for (r, L), s in table.items():
        for hi in range(1 << (15 - L)):
            t[r | hi << L] = (s, L)
    return t


def bgzf_blocks(data):
    o = 0
    while o + 18 <= len(data):
        bsize = struct.unpack_from("<H", data, o + 16)[0] + 1
        yield bytes(data[o + 18:o + bsize - 8])
        o += bsize


def spec(v, nbits, p, lt, dt, truth, limit):
    """tokens decoded from bit p until a true token start (or an invalid code / the limit)"""
    n = 0
    while n < limit and p < nbits - 64:
        if p in truth:
            return n, True
        x = (v >> p) & 0x7fff
        e = lt[x]
        if e is None:
            return n, False
        s, L = e
        p += L
        if s >= 257:
            if s > 285:
                return n, False
            i = s - 257
            p += LEXT[i]
            e = dt[(v >> p) & 0x7fff]
            if e is None or e[0] > 29:
                return n, False
            p += e[1] + DEXT[e[0]]
        n += 1
    return n, p in truth


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mb", type=float, nargs="?", default=2.0)
    ap.add_argument("--starts", type=int, default=64)
    a = ap.parse_args()
    data = bytes(genbam.generate(target_bytes=int(a.mb * 1e6), threads=4, seed=3))
    rng = random.Random(1)
    nblk = 0
    ndb = {}
    first_frac = []
    sync = []
    fails = 0
    for raw in bgzf_blocks(data):
        if len(raw) < 64:
            continue
        blocks, toks, out = trace(raw)
        nblk += 1
        ndb[len(blocks)] = ndb.get(len(blocks), 0) + 1
        tot = sum(b.get("symbols", 0) for b in blocks)
        first_frac.append(blocks[0].get("symbols", 0) / max(tot, 1))
        if nblk % 4:
            continue
        v = int.from_bytes(raw + bytes(16), "little")
        nbits = 8 * len(raw)
        for bi, b in enumerate(blocks):
            if b["type"] == 0:
                continue
            bits = Bits(raw)
            # rebuild this block's tables from the trace's header (re-decode the header)
            bits.p = b["bit"] + 3
            if b["type"] == 1:
                ll = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
                dl = [5] * 32
            else:
                from deflate_trace import ORDER, decode_sym
                hlit, hdist, hclen = bits.get(5) + 257, bits.get(5) + 1, bits.get(4) + 4
                cl = [0] * 19
                for i in range(hclen):
                    cl[ORDER[i]] = bits.get(3)
                ct = canon(cl)
                lens = []
                while len(lens) < hlit + hdist:
                    s, _ = decode_sym(bits, ct)
                    if s < 16:
                        lens.append(s)
                    elif s == 16:
                        lens += [lens[-1]] * (3 + bits.get(2))
                    elif s == 17:
                        lens += [0] * (3 + bits.get(3))
                    else:
                        lens += [0] * (11 + bits.get(7))
                ll, dl = lens[:hlit], lens[hlit:]
            lt, dt = lut(canon(ll)), lut(canon(dl))
            s0, s1 = b["bit"] + b["hdr_bits"], b["end_bit"]
            truth = set(t[0] for t in toks if s0 <= t[0] < s1)
            for _ in range(a.starts // len(blocks)):
                p = rng.randrange(s0, max(s0 + 1, s1 - 2000))
                n, ok = spec(v, nbits, p, lt, dt, truth, 4000)
                if ok:
                    sync.append(n)
                else:
                    fails += 1
    print("BGZF blocks %d  DEFLATE blocks per BGZF block %s" % (nblk, sorted(ndb.items())))
    ff = sorted(first_frac)
    print("first DEFLATE block's share of symbols: median %.2f  p10 %.2f" % (ff[len(ff) // 2], ff[len(ff) // 10]))
    sync.sort()
    if sync:
        print("speculative starts %d (+%d hit an invalid code): tokens to sync median %d  p90 %d  p99 %d  max %d" %
              (len(sync), fails, sync[len(sync) // 2], sync[int(len(sync) * .9)], sync[int(len(sync) * .99)], sync[-1]))


if __name__ == "__main__":
    main()
