"""Device inflate of one window's blocks at every 16-byte misalignment of the output buffer
(a leading copy of a short block shifts the rest), each block against zlib: first differing
offset per block."""
import os
import struct
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hadoop-bam_amd")]
import numpy as np  # noqa: E402

from hadoop_bam import _lib  # noqa: E402

ctx = _lib.Context(0)
for name in sys.argv[1:]:
    w = np.fromfile(os.path.join(ROOT, "tests", "golden", name), np.uint8)
    bw = w.tobytes()
    p = bw.find(b"\x1f\x8b\x08\x04")
    blocks = []
    while p + 18 <= len(bw) and bw[p:p + 4] == b"\x1f\x8b\x08\x04":
        bs = struct.unpack("<H", bw[p + 16:p + 18])[0] + 1
        if p + bs > len(bw):
            break
        c_, i_ = struct.unpack("<II", bw[p + bs - 8:p + bs])
        blocks.append((p, bs, i_, c_))
        p += bs
    short = [b for b in blocks if b[2] % 16]
    ref = {b[0]: zlib.decompressobj(-15).decompress(bw[b[0] + 18:b[0] + b[1] - 8]) for b in blocks}
    for lead in range(0, 16):
        # leading blocks whose ISIZE sum to `lead` mod 16: the short block k times
        lst = []
        if lead:
            k = next(k for k in range(1, 17) if (k * short[0][2]) % 16 == lead)
            lst = [short[0]] * k
        lst = lst + blocks
        B = {"coff": np.array([b[0] for b in lst], np.uint64), "clen": np.array([b[1] for b in lst], np.uint32),
             "isize": np.array([b[2] for b in lst], np.uint32), "crc": np.array([b[3] for b in lst], np.uint32)}
        rc, u, off, st = ctx.inflate(w, B, check_crc=True)
        bad = []
        for j, b in enumerate(lst):
            got = u[int(off[j]):int(off[j + 1])].tobytes()
            if got != ref[b[0]]:
                d = next(i for i in range(len(got)) if got[i] != ref[b[0]][i])
                bad.append((j, b[0], b[2], int(st[j]), d, got[d:d + 8].hex(), ref[b[0]][d:d + 8].hex()))
        print(name, "misalign", lead, "bad blocks", len(bad), bad[:4], flush=True)
