"""Token trace of a raw DEFLATE stream (pure Python, RFC 1951), for diagnosing the device
Huffman pass and for sizing its tables: every symbol's starting bit, output position, kind
(literal / match / end of block) and code length; every DEFLATE block's header position,
type and code-length histogram.

    python tools/deflate_trace.py BLOCK.bgzf [--at OUTPOS] [--bit BITPOS] [--stats]
"""
import argparse
import zlib

ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115,
         131, 163, 195, 227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537,
         2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


class Bits:
    def __init__(self, data):
        self.v = int.from_bytes(data, "little")
        self.n = 8 * len(data)
        self.p = 0

    def get(self, k):
        if self.p + k > self.n:
            raise EOFError("stream ends at bit %d" % self.p)
        x = (self.v >> self.p) & ((1 << k) - 1)
        self.p += k
        return x


def canon(lengths):
    """(code, length) -> symbol, with codes as read LSB-first (bit-reversed canonical codes)."""
    cnt = [0] * 16
    for L in lengths:
        cnt[L] += 1
    cnt[0] = 0
    code, nxt = 0, [0] * 16
    for L in range(1, 16):
        code = (code + cnt[L - 1]) << 1
        nxt[L] = code
    table = {}
    for s, L in enumerate(lengths):
        if L:
            c = nxt[L]
            nxt[L] += 1
            r = int("{:0{w}b}".format(c, w=L)[::-1], 2)
            table[(r, L)] = s
    return table


def decode_sym(bits, table):
    code = 0
    for L in range(1, 16):
        code |= bits.get(1) << (L - 1)
        s = table.get((code, L))
        if s is not None:
            return s, L
    raise ValueError("invalid code at bit %d" % bits.p)


def trace(raw):
    """raw DEFLATE -> (blocks, tokens); token = (bit, outpos, kind, value, code_bits, total_bits)."""
    bits = Bits(raw)
    out = 0
    blocks, toks = [], []
    while True:
        hb = bits.p
        last = bits.get(1)
        typ = bits.get(2)
        info = {"bit": hb, "out": out, "type": typ, "last": last}
        if typ == 0:
            bits.p = (bits.p + 7) & ~7
            ln = bits.get(16)
            bits.get(16)
            for _ in range(ln):
                toks.append((bits.p, out, "lit", bits.get(8), 8, 8))
                out += 1
            info["len"] = ln
            blocks.append(info)
        else:
            if typ == 1:
                ll = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
                dl = [5] * 32
            else:
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
                info.update(hlit=hlit, hdist=hdist, hclen=hclen)
            info["hdr_bits"] = bits.p - hb
            info["ll_hist"] = [sum(1 for x in ll if x == L) for L in range(16)]
            info["d_hist"] = [sum(1 for x in dl if x == L) for L in range(16)]
            lt, dt = canon(ll), canon(dl)
            nsym = 0
            while True:
                sb = bits.p
                s, L = decode_sym(bits, lt)
                nsym += 1
                if s < 256:
                    toks.append((sb, out, "lit", s, L, L))
                    out += 1
                elif s == 256:
                    toks.append((sb, out, "eob", 0, L, L))
                    break
                else:
                    i = s - 257
                    ln = LBASE[i] + bits.get(LEXT[i])
                    ds, dL = decode_sym(bits, dt)
                    dist = DBASE[ds] + bits.get(DEXT[ds])
                    toks.append((sb, out, "match", (ln, dist), (L, LEXT[i], dL, DEXT[ds]), bits.p - sb))
                    out += ln
            info["symbols"] = nsym
            info["end_bit"] = bits.p
            blocks.append(info)
        if last:
            break
    return blocks, toks, out


def bgzf_payload(member):
    xlen = member[10] | member[11] << 8
    return member[12 + xlen:len(member) - 8]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--at", type=int, default=None, help="print the tokens around this output position")
    ap.add_argument("--bit", type=int, default=None, help="print the tokens around this stream bit")
    ap.add_argument("--stats", action="store_true")
    a = ap.parse_args()
    member = open(a.path, "rb").read()
    raw = bgzf_payload(member)
    blocks, toks, out = trace(raw)
    ref = zlib.decompress(raw, -15)
    assert out == len(ref), (out, len(ref))
    print("stream bits %d, output %d bytes, %d DEFLATE blocks, %d tokens" % (8 * len(raw), out, len(blocks), len(toks)))
    for b in blocks:
        print("  block", {k: v for k, v in b.items() if k not in ("ll_hist", "d_hist")})
        if a.stats and "ll_hist" in b:
            print("    lit/len lengths", b["ll_hist"], " dist lengths", b["d_hist"])
    idx = None
    if a.at is not None:
        idx = max(i for i, t in enumerate(toks) if t[1] <= a.at)
    elif a.bit is not None:
        idx = max(i for i, t in enumerate(toks) if t[0] <= a.bit)
    if idx is not None:
        for i in range(max(0, idx - 6), min(len(toks), idx + 6)):
            print("%s tok %6d bit %7d out %6d %-5s %s codebits %s total %d" %
                  ("=>" if i == idx else "  ", i, toks[i][0], toks[i][1], toks[i][2], toks[i][3], toks[i][4], toks[i][5]))


if __name__ == "__main__":
    main()
