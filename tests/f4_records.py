"""Synthetic BAM records for the f-4 consumer tests: SAMRecordWritable payloads
(block_size + record, SAM/BAM v1 §4.2 layout) built directly, so the edge cases the consumers
branch on can be placed exactly: CIGARs with every op, op codes > 8, records without a range,
read names sharing prefixes / of every length / with bytes >= 0x80, pairs of every mapped /
unmapped combination, secondaries, >2 primaries per name, MQ / MC and integer tags of every type.
"""
import struct

import numpy as np

OPS = "MIDNSHP=X"


def aux_int(tag, typ, v):
    fmt = {"c": "<b", "C": "<B", "s": "<h", "S": "<H", "i": "<i", "I": "<I"}[typ]
    return tag.encode() + typ.encode() + struct.pack(fmt, v)


def aux_z(tag, s):
    return tag.encode() + b"Z" + s.encode() + b"\0"


def record(name=b"r", flag=0, ref=0, pos=0, mapq=60, cigar=((10, 0),), l_seq=10, aux=b"",
           nref=-1, npos=-1, tlen=0, bin_=4681, qual_absent=False, seed=0, raw_ops=None):
    """One payload.  cigar: (len, op) pairs; raw_ops: u32 CIGAR words as given (garbage ops)."""
    rng = np.random.default_rng(seed)
    words = list(raw_ops) if raw_ops is not None else [(ln << 4) | op for ln, op in cigar]
    seq = bytes(rng.integers(0, 256, (l_seq + 1) // 2, dtype=np.uint8))
    qual = b"\xff" * l_seq if qual_absent else bytes(rng.integers(0, 42, l_seq, dtype=np.uint8))
    var = name + b"\0" + b"".join(struct.pack("<I", w) for w in words) + seq + qual + aux
    fixed = struct.pack("<iiBBHHHiiii", ref, pos, len(name) + 1, mapq, bin_, len(words), flag, l_seq,
                        nref, npos, tlen)
    body = fixed + var
    return struct.pack("<i", len(body)) + body


def pack(recs):
    """payload bytes + offsets (u64[n+1])"""
    off = np.zeros(len(recs) + 1, np.uint64)
    off[1:] = np.cumsum([len(r) for r in recs])
    return np.frombuffer(b"".join(recs), np.uint8).copy(), off


def summarize_edge_records():
    """Records covering SummarizeRecordReader's branches (Summarize.java:693-755)."""
    R = []
    R.append(record(b"a", flag=0x10, ref=3, pos=99,
                    cigar=((5, 4), (10, 0), (3, 1), (10, 0), (2, 2), (5, 0), (4, 3), (6, 0), (2, 5)), l_seq=41))
    R.append(record(b"b", flag=4, ref=1, pos=10))                      # unmapped: skipped
    R.append(record(b"c", flag=0, ref=-1, pos=10))                     # unplaced: skipped
    R.append(record(b"d", flag=0, ref=2, pos=-2))                      # start < 0: skipped
    R.append(record(b"e", flag=0, ref=2, pos=-1, cigar=((7, 0),), l_seq=7))  # start 0: kept
    R.append(record(b"f", flag=0, ref=0, pos=5, cigar=((3, 7), (2, 8), (4, 6), (1, 0)), l_seq=6))
    R.append(record(b"g", flag=0, ref=24, pos=0x7ffffff0, cigar=((100, 0),), l_seq=100))  # int wrap
    R.append(record(b"h", flag=0, ref=5, pos=1000, cigar=((20, 0), (30, 2), (20, 0)), l_seq=40))
    R.append(record(b"i", flag=0x10, ref=5, pos=1000, cigar=((1, 2), (5, 0), (1, 3), (5, 0)), l_seq=10))
    return R


def overrun_record(field="cigar"):
    """A mapped record whose n_cigar (field 'cigar') or l_seq ('seq') claims more bytes than its
    block_size holds: decode hands it out with status OK and layout_ok 0, and htsjdk throws only
    when the field is read (the consumers read such fields past the record)."""
    b = bytearray(record(b"ovr", flag=0x41, ref=1, pos=60, cigar=((10, 0),), l_seq=10))
    if field == "cigar":
        struct.pack_into("<H", b, 16, 5000)     # n_cigar (payload offset 4 + 12)
    else:
        struct.pack_into("<i", b, 20, 1 << 20)  # l_seq (payload offset 4 + 16)
    return bytes(b)


def summarize_error_records(kind):
    """kind 'op': a CIGAR op code 9 in a mapped record (IllegalArgumentException); 'empty': a mapped
    record whose CIGAR has no M/=/X (ranges.get(0) -> IndexOutOfBoundsException); 'overrun': a
    mapped record whose CIGAR lies past its block_size (getCigar's read throws)."""
    R = summarize_edge_records()
    if kind == "overrun":
        R.insert(5, overrun_record("cigar"))
    elif kind == "op":
        R.insert(5, record(b"x", flag=0, ref=1, pos=50, raw_ops=[(10 << 4) | 0, (3 << 4) | 9]))
    else:
        R.insert(5, record(b"x", flag=0, ref=1, pos=50, cigar=((5, 4), (3, 1)), l_seq=8))
    return R


def names_records(n=600, seed=11):
    """Read names exercising Text order: shared prefixes, every length 0..40, 8-byte chunk
    boundaries, bytes >= 0x80, exact duplicates."""
    rng = np.random.default_rng(seed)
    R = []
    stems = [b"", b"A", b"AB", b"ABCDEFGH", b"ABCDEFGHI", b"ABCDEFGH\x80", b"\x7fZ", b"\xff\xfe",
             b"SRR000.1", b"SRR000.10", b"SRR000.2", b"r" * 40]
    for i in range(n):
        if i < len(stems):
            nm = stems[i]
        elif rng.random() < 0.3:
            nm = stems[int(rng.integers(0, len(stems)))]
        else:
            L = int(rng.integers(0, 41))
            nm = bytes(rng.choice(np.frombuffer(b"ACGT:_.#\x80\xfe", np.uint8), L))
        nm = nm.replace(b"\0", b"A")
        R.append(record(nm, flag=int(rng.integers(0, 4096)) & ~0x4, ref=int(rng.integers(0, 5)),
                        pos=int(rng.integers(0, 10**6)), seed=i))
    return R


def fixmate_records(seed=5):
    """Key groups for FixMateReducer (FixMate.java:230-277): pairs of every mapped / unmapped
    combination, with and without MQ / MC / integer tags of every type; secondaries before,
    between and after primaries; single primaries; three and four primaries; a primary followed
    only by secondaries (the quirk: mated with the last one, written twice); zero-length names."""
    rng = np.random.default_rng(seed)
    R = []
    tags_all = (aux_z("RG", "grp1") + aux_int("NM", "C", 3) + aux_int("AS", "i", 140) +
                aux_int("XS", "s", -5) + aux_int("XB", "I", 70000) + aux_int("XC", "S", 300) +
                aux_int("XD", "c", -100) + aux_z("MC", "150M") + aux_int("MQ", "C", 17) +
                b"XFf" + struct.pack("<f", 1.5) + b"XHH" + b"1AE3\0" + b"XAA" + b"Q" +
                b"XBBs" + struct.pack("<I", 3) + struct.pack("<hhh", 1, -2, 3))
    g = 0

    def nm():
        return b"pair%05d" % g

    # both mapped, same reference, forward/reverse, equal 5' ends, with tags
    for case in range(40):
        g += 1
        ref = int(rng.integers(0, 3))
        p1, p2 = int(rng.integers(0, 5000)), int(rng.integers(0, 5000))
        if case % 5 == 0:
            p2 = p1
        ref2 = ref if case % 7 else ref + 1
        f1 = 1 | 0x40 | (0x10 if case % 2 else 0)
        f2 = 1 | 0x80 | (0x10 if case % 3 == 0 else 0)
        aux1 = tags_all if case % 4 == 0 else aux_int("NM", "i", case)
        aux2 = aux_z("MC", "10M") if case % 3 == 0 else b""
        R.append(record(nm(), flag=f1, ref=ref, pos=p1, mapq=int(rng.integers(0, 256)),
                        cigar=((20, 0), (2, 2), (20, 0)), l_seq=40, aux=aux1, seed=g))
        R.append(record(nm(), flag=f2, ref=ref2, pos=p2, mapq=int(rng.integers(0, 256)),
                        cigar=((3, 4), (37, 0)), l_seq=41, aux=aux2, seed=g + 1000,
                        qual_absent=(case % 6 == 0)))
    # one mapped, one unmapped (either order); both unmapped
    for case in range(20):
        g += 1
        fa = 1 | 0x40 | (4 if case % 2 else 0) | (0x10 if case % 3 == 0 else 0)
        fb = 1 | 0x80 | (0 if case % 2 else 4) | (0x10 if case % 4 == 0 else 0)
        if case >= 14:
            fa |= 4
            fb |= 4
        R.append(record(nm(), flag=fa, ref=1, pos=777 + case, cigar=((30, 0),), l_seq=30,
                        aux=aux_int("MQ", "c", 5) if case % 5 == 0 else b"", seed=g))
        R.append(record(nm(), flag=fb, ref=2 if case % 2 else -1, pos=-1 if case % 2 == 0 else 50,
                        cigar=((30, 0),), l_seq=31, seed=g + 2000))
    # secondaries in every place, singles, >2 primaries, the quirk
    shapes = ["SPSP", "PSSP", "PS", "PSS", "P", "S", "SS", "PPP", "PPPP", "PSPSP", "SPPS"]
    for case, shape in enumerate(shapes * 3):
        g += 1
        for j, ch in enumerate(shape):
            fl = 1 | (0x100 if ch == "S" else 0) | (4 if (case + j) % 5 == 0 else 0)
            R.append(record(nm(), flag=fl, ref=int(rng.integers(0, 3)), pos=int(rng.integers(0, 9000)),
                            cigar=((15, 0), (1, 1), (14, 0)), l_seq=30,
                            aux=aux_int("NM", "S", j) + aux_z("MC", "30M"), seed=g * 10 + j))
    # empty names share one key group
    for j in range(3):
        R.append(record(b"", flag=1 | (0x40 if j == 0 else 0x80), ref=0, pos=10 * j, seed=9000 + j))
    order = rng.permutation(len(R))  # the shuffle sees them in any input order
    return [R[i] for i in order]
