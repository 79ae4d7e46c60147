"""BGZFBlockIndexer / BGZFBlockIndex / BGZFSplitFileInputFormat.

CPU: the oracle restatement (oracle/hbam_oracle.c or_bgzf_block_index) against an independent
pure-Python restatement of util/BGZFBlockIndexer.java:97-181 and against the block table, incl.
blocks with a foreign extra subfield and a truncated final block; the index reader
(util/BGZFBlockIndex.java:50-69) and the indexed split path
(util/BGZFSplitFileInputFormat.java:85-122).
GPU: hbam_bgzf_block_index bit-exact against the oracle, incl. the int `pos` wrap past 2 GiB.
"""
import io
import os
import struct

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def py_bgzf_block_index(f, g):
    """util/BGZFBlockIndexer.java:97-181 line by line (FileInputStream semantics: reads at or
    past EOF return nothing, skip moves past EOF)."""
    f = bytes(f)
    at, pos, out, i = 0, 0, [], 0

    def read(k):
        nonlocal at
        b = f[at:at + k] if at < len(f) else b""
        at += len(b)
        return b

    while True:
        b = read(4)
        if len(b) != 4:
            if len(b) == 0:
                break
            raise IOError("too short")
        if struct.unpack(">I", b)[0] != 0x1F8B0804:
            raise IOError("bad magic")
        b = read(8)
        if len(b) != 8:
            raise IOError("no XLEN")
        xlen = struct.unpack("<H", b[6:8])[0]
        off, found = 0, False
        while off < xlen:
            b = read(4)
            if len(b) != 4:
                raise IOError("EOF in subfields")
            off += 4
            if (struct.unpack(">I", b)[0] & ~0xFF) & 0xFFFFFFFF == 0x42430200:
                b = read(2)
                if len(b) != 2:
                    raise IOError("missing BSIZE")
                off += 2
                bsize = struct.unpack("<H", b)[0]
                skip = (xlen - off) + (bsize - xlen - 19) + 8
                if skip > 0:
                    at += skip
                pos = (pos + bsize + 1) & 0xFFFFFFFF
                found = True
                break
            slen = struct.unpack("<H", b[2:4])[0]
            at += slen
            off += slen
        if not found:
            raise IOError("block without BGZF subfield")
        i += 1
        if i == g:
            i = 0
            sp = pos - (1 << 32) if pos >= (1 << 31) else pos
            out.append(sp & 0xFFFFFFFFFFFF)
    out.append(len(f) & 0xFFFFFFFFFFFF)
    return out


def _load(name):
    return np.fromfile(os.path.join(GOLDEN, name), dtype=np.uint8)


def _with_extra_subfield(data, oracle_mod, every=2):
    """Rewrite every `every`-th block with a 4-byte foreign subfield ('XY', SLEN 0) before
    BC (XLEN 10, BSIZE+4): legal gzip that the reference's subfield loop must step over."""
    blk = oracle_mod.scan_blocks(data)
    d = bytes(data)
    parts = []
    for i, (c, l) in enumerate(zip(blk["coff"], blk["clen"])):
        c, l = int(c), int(l)
        b = d[c:c + l]
        if i % every == 0:
            bsize = struct.unpack("<H", b[16:18])[0] + 4
            b = b[:10] + struct.pack("<H", 10) + b"XY\x00\x00" + b"BC\x02\x00" + \
                struct.pack("<H", bsize) + b[18:]
        parts.append(b)
    return np.frombuffer(b"".join(parts), dtype=np.uint8)


@pytest.mark.parametrize("g", [1, 2, 3, 7, 100, 100000])
def test_oracle_matches_python_restatement(oracle_mod, small_bam, g):
    want = py_bgzf_block_index(small_bam, g)
    got = oracle_mod.bgzf_block_index(small_bam, g)
    assert list(map(int, got)) == want


def test_oracle_entries_are_block_ends(oracle_mod, small_bam):
    blk = oracle_mod.scan_blocks(small_bam)
    ends = [int(c) + int(l) for c, l in zip(blk["coff"], blk["clen"])]
    for g in (1, 5):
        got = list(map(int, oracle_mod.bgzf_block_index(small_bam, g)))
        assert got[:-1] == ends[g - 1::g]
        assert got[-1] == len(small_bam)


def test_oracle_steps_over_foreign_subfields(oracle_mod, small_bam):
    d = _with_extra_subfield(small_bam, oracle_mod)
    for g in (1, 3):
        want = py_bgzf_block_index(d, g)
        assert list(map(int, oracle_mod.bgzf_block_index(d, g))) == want
    # offsets still land on the (shifted) block boundaries
    got = list(map(int, oracle_mod.bgzf_block_index(d, 1)))
    pos, b = 0, bytes(d)
    for e in got[:-1]:
        assert b[e:e + 4] == b"\x1f\x8b\x08\x04" or e == len(b)
        pos = e
    assert pos == len(b)


def test_oracle_error_and_edge_cases(oracle_mod, small_bam):
    assert list(map(int, oracle_mod.bgzf_block_index(np.zeros(0, np.uint8), 1))) == [0]
    bad = small_bam.copy()
    bad[0] = 0
    assert oracle_mod.bgzf_block_index(bad, 1) == oracle_mod.OR_EIO
    # truncated final block: FileInputStream.skip runs past EOF, so the block still counts
    t = small_bam[:-10]
    got = list(map(int, oracle_mod.bgzf_block_index(t, 1)))
    assert got == py_bgzf_block_index(t, 1)
    assert got[-2] == len(small_bam) and got[-1] == len(t)
    # trailing 1..3 bytes: "too short, no ID/CM/FLG"
    assert oracle_mod.bgzf_block_index(np.concatenate([small_bam, small_bam[:2]]), 1) == oracle_mod.OR_EIO


def test_index_reader_roundtrip_and_order(oracle_mod, small_bam):
    from hadoop_bam import BGZFBlockIndex
    from hadoop_bam.formats import IOException
    offs = list(map(int, oracle_mod.bgzf_block_index(small_bam, 2)))
    raw = b"".join(struct.pack(">q", o)[2:] for o in offs)
    idx = BGZFBlockIndex(io.BytesIO(raw))
    assert idx.size() == len(set(offs) | {0})
    assert idx.fileSize() == len(small_bam)
    assert idx.prevBlock(0) == 0 and idx.nextBlock(0) == offs[0]
    assert idx.prevBlock(offs[1] + 5) == offs[1]
    assert idx.nextBlock(len(small_bam)) is None
    with pytest.raises(IOException):
        BGZFBlockIndex(io.BytesIO(raw[6:12] + raw[:6]))
    with pytest.raises(IOException):
        BGZFBlockIndex(io.BytesIO(b""))


def test_indexed_splits(tmp_path, oracle_mod, small_bam):
    """BGZFSplitFileInputFormat.addIndexedSplits over a .bgzfi written from the oracle: split
    starts snap back to indexed blocks, inner ends forward, the last end back."""
    from hadoop_bam import BGZFSplitFileInputFormat, FileSplit
    path = str(tmp_path / "x.bam")
    small_bam.tofile(path)
    offs = list(map(int, oracle_mod.bgzf_block_index(small_bam, 3)))
    with open(path + ".bgzfi", "wb") as f:
        f.write(b"".join(struct.pack(">q", o)[2:] for o in offs))
    n = len(small_bam)
    step = n // 5 + 1
    splits = [FileSplit(path, s, min(step, n - s)) for s in range(0, n, step)]
    got = BGZFSplitFileInputFormat().getSplits(splits)
    table = sorted(set(offs) | {0})
    import bisect

    def floor(x):
        return table[bisect.bisect_right(table, x) - 1]

    def higher(x):
        return table[bisect.bisect_right(table, x)]
    assert len(got) == len(splits)
    for j, (s, o) in enumerate(zip(splits, got)):
        st, en = s.getStart(), s.getStart() + s.getLength()
        be = floor(en) if j == len(splits) - 1 else higher(en)
        assert (o.getStart(), o.getStart() + o.getLength()) == (floor(st), be)


# ---- device ---------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("fname", ["small_pe.bam", "edge_uniform_long.bam", "edge_unsorted_l1.bam"])
@pytest.mark.parametrize("g", [1, 2, 3, 7, 1000, 100000])
def test_device_block_index_matches_oracle(gpu_ctx, oracle_mod, fname, g):
    data = _load(fname)
    want = oracle_mod.bgzf_block_index(data, g)
    rc, got = gpu_ctx.bgzf_block_index(data, g)
    assert rc == 0, gpu_ctx.last_error()
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_device_block_index_edges(gpu_ctx, oracle_mod, small_bam):
    rc, got = gpu_ctx.bgzf_block_index(np.zeros(0, np.uint8), 1)
    assert rc == 0 and list(got) == [0]
    bad = small_bam.copy()
    bad[0] = 0
    rc, _ = gpu_ctx.bgzf_block_index(bad, 1)
    assert rc == -1  # IOException
    # documented deviation: a truncated final block raises IOException here,
    # where the reference's FileInputStream.skip past EOF still counts it
    rc, _ = gpu_ctx.bgzf_block_index(small_bam[:-10], 1)
    assert rc == -1


@pytest.mark.gpu
def test_indexer_writes_reference_bytes(tmp_path, gpu_ctx, oracle_mod, small_bam):
    from hadoop_bam import BGZFBlockIndexer, BGZFSplitFileInputFormat, FileSplit
    path = str(tmp_path / "y.bam")
    small_bam.tofile(path)
    raw = BGZFBlockIndexer(4, ctx=gpu_ctx).index(path)
    want = b"".join(struct.pack(">q", int(o))[2:] for o in oracle_mod.bgzf_block_index(small_bam, 4))
    assert raw == want and open(path + ".bgzfi", "rb").read() == want
    # probabilistic path (no index): split starts are the device BGZFSplitGuesser's
    os.remove(path + ".bgzfi")
    n = len(small_bam)
    splits = [FileSplit(path, s, min(40000, n - s)) for s in range(0, n, 40000)]
    got = BGZFSplitFileInputFormat().getSplits(splits)
    for s, o in zip(splits, got):
        st, en = s.getStart(), s.getStart() + s.getLength()
        assert o.getStart() == oracle_mod.guess_bgzf_block_start(small_bam, st, en)[0]
        assert o.getStart() + o.getLength() == en


@pytest.mark.gpu
def test_device_block_index_int_wrap_past_2gib(gpu_ctx, oracle_mod, genbam):
    """Files past 2^31 bytes: the reference's int `pos` wraps; entries must match bit for bit."""
    data = np.asarray(genbam.generate(target_bytes=int(2.2e9), seed=5, threads=16, level=1))
    assert len(data) > (1 << 31)
    g = 64
    want = oracle_mod.bgzf_block_index(data, g)
    rc, got = gpu_ctx.bgzf_block_index(data, g)
    assert rc == 0, gpu_ctx.last_error()
    assert np.array_equal(got, want)
    assert int(got[-2]) > (1 << 47)  # a wrapped (sign-extended) entry
