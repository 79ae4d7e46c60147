"""Blocks file for the CPU model (tools/cpu_model/tok_model.cpp): every BGZF block of the eight
generated BAMs tools/check_inflate_crc.py checks on the device (same seeds, quality models and
compression levels), at a small size, as raw DEFLATE bytes + the bytes zlib inflates them to.

format: "HBTM" u32 magic, u32 block count, then per block: u32 raw length, u32 ISIZE, raw bytes,
inflated bytes.

usage: make_blocks.py OUT [MB_PER_FILE]
"""
import os
import struct
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import genbam  # noqa: E402

CASES = [dict(seed=s) for s in (3, 4, 5, 6)] + [dict(seed=7, uniform_qual=1), dict(seed=8, level=1),
                                                 dict(seed=9, level=9), dict(seed=10, level=6, uniform_qual=1)]


def bgzf_blocks(data):
    o = 0
    while o + 18 <= len(data):
        assert data[o:o + 4] == b"\x1f\x8b\x08\x04", o
        bsize = struct.unpack_from("<H", data, o + 16)[0] + 1
        raw = bytes(data[o + 18:o + bsize - 8])
        isize = struct.unpack_from("<I", data, o + bsize - 4)[0]
        yield raw, isize
        o += bsize


def main():
    out = sys.argv[1]
    mb = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
    recs = []
    for kw in CASES:
        data = bytes(genbam.generate(target_bytes=int(mb * 1e6), threads=4, **kw))
        for raw, isize in bgzf_blocks(data):
            u = zlib.decompress(raw, -15) if isize else b""
            assert len(u) == isize
            recs.append((raw, u))
    with open(out, "wb") as f:
        f.write(struct.pack("<II", 0x4d544248, len(recs)))
        for raw, u in recs:
            f.write(struct.pack("<II", len(raw), len(u)))
            f.write(raw)
            f.write(u)
    print("%d blocks -> %s" % (len(recs), out))


if __name__ == "__main__":
    main()
