"""BAM output: the device BGZF compressor and the writer classes.

Parity is on the inflated bytes (the compressed bytes are the device
compressor's, not zlib's): every member inflates with zlib (the JDK's inflater) to the input,
its CRC32 and ISIZE are right, the member chain is the one htsjdk's reader walks, and a BAM
written by BAMRecordWriter / the Sort output path reads back — through the oracle's
BAMRecordReader — to exactly the records written, in order."""
import os
import struct
import zlib

import numpy as np
import pytest

from conftest import GOLDEN


def _members(comp):
    """Walk BGZF members -> list of (inflated bytes, isize, crc_ok, bsize)."""
    out, p = [], 0
    while p < len(comp):
        assert comp[p:p + 4] == b"\x1f\x8b\x08\x04"
        assert comp[p + 10:p + 16] == b"\x06\x00BC\x02\x00"
        bs = struct.unpack_from("<H", comp, p + 16)[0] + 1
        crc, isz = struct.unpack_from("<II", comp, p + bs - 8)
        d = zlib.decompressobj(-15)
        u = d.decompress(comp[p + 18:p + bs - 8])
        assert d.eof and not d.unused_data
        out.append((u, isz, zlib.crc32(u) == crc, bs))
        p += bs
    assert p == len(comp)
    return out


# ---- CPU: header serialization --------------------------------------------------------------
def test_header_bytes_round_trip():
    """SAMFileHeader.to_bam_bytes is BAMRecordWriter.writeHeader's layout: the inflated header
    of a BAM parses and re-serializes to the same bytes."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(GOLDEN), "..", "oracle"))
    from hadoop_bam.output import SAMFileHeader
    data = open(os.path.join(GOLDEN, "small_pe.bam"), "rb").read()
    u, p = b"", 0
    while len(u) < 1 << 20 and p < len(data):
        bs = struct.unpack_from("<H", data, p + 16)[0] + 1
        u += zlib.decompressobj(-15).decompress(data[p + 18:p + bs - 8])
        p += bs
    h = SAMFileHeader.from_bam_bytes(u)
    b = h.to_bam_bytes()
    assert u[:len(b)] == b
    assert len(h.refs) > 0 and h.text.startswith(b"@")


def test_set_sort_order():
    from hadoop_bam.output import SAMFileHeader
    h = SAMFileHeader(b"@HD\tVN:1.4\tSO:unsorted\n@SQ\tSN:c1\tLN:10\n", [(b"c1", 10)])
    h.setSortOrder("coordinate")
    assert h.text.split(b"\n")[0] == b"@HD\tVN:1.4\tSO:coordinate"
    h2 = SAMFileHeader(b"@SQ\tSN:c1\tLN:10\n", [(b"c1", 10)])
    h2.setSortOrder("coordinate")
    assert h2.text.startswith(b"@HD\tVN:1.4\tSO:coordinate\n@SQ")


def test_mergeable_work_file_name():
    from hadoop_bam.output import get_mergeable_work_file
    assert get_mergeable_work_file("/w", "pre-", "-post", "sort", 7, "bam") == "/w/pre-sort-post-000007.bam"


# ---- GPU: the compressor ------------------------------------------------------------------
def _inputs():
    rng = np.random.default_rng(9)
    u = b""
    data = open(os.path.join(GOLDEN, "small_pe.bam"), "rb").read()
    p = 0
    while p < len(data):
        bs = struct.unpack_from("<H", data, p + 16)[0] + 1
        u += zlib.decompressobj(-15).decompress(data[p + 18:p + bs - 8])
        p += bs
    # Fibonacci byte counts (1, 1, 2, 3, 5, ...) in random order: the Huffman tree of the
    # literals is deeper than 15, so the lit/len code must be length-limited (an
    # under-repaired limit left the code over-subscribed and zlib rejected the member)
    fib = [1, 1]
    while len(fib) < 22:
        fib.append(fib[-1] + fib[-2])
    fib_bytes = np.repeat(np.arange(22, dtype=np.uint8) * 11, fib)
    rng.shuffle(fib_bytes)
    # skewed random blocks: per block a Pareto-distributed byte histogram
    skew = []
    for _ in range(6):
        w = rng.pareto(0.6, 256) + 1e-3
        skew.append(rng.choice(256, 65280, p=w / w.sum()).astype(np.uint8))
    return {
        "fib_literals": fib_bytes.tobytes(),
        "skewed": np.concatenate(skew).tobytes(),
        "one": b"A",
        "small": bytes(range(256)) * 3,
        "block": rng.integers(0, 4, 65280, dtype=np.uint8).tobytes(),
        "block+1": rng.integers(0, 4, 65281, dtype=np.uint8).tobytes(),
        "random": rng.integers(0, 256, 3 * 65280 + 17, dtype=np.uint8).tobytes(),
        "zeros": bytes(200000),
        "period3": b"ACG" * 70000,
        "bam_stream": u,
    }


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(_inputs().keys()))
@pytest.mark.parametrize("block_size", [0, 4096])
def test_bgzf_compress_inflates_back(gpu_ctx, name, block_size):
    src = _inputs()[name]
    comp = gpu_ctx.bgzf_compress(src, block_size).tobytes()
    ms = _members(comp)
    bs = block_size or 65280
    assert len(ms) == (len(src) + bs - 1) // bs
    assert b"".join(m[0] for m in ms) == src
    for u, isz, crc_ok, bsz in ms:
        assert isz == len(u) <= bs and crc_ok and bsz <= 65536


@pytest.mark.gpu
def test_bgzf_compress_from_device_and_reads_on_device(gpu_ctx, oracle_mod):
    """Device source -> device destination; the device's own reader (scan + inflate with CRC
    check) and the oracle both walk the result."""
    import torch
    src = _inputs()["bam_stream"]
    d = torch.from_numpy(np.frombuffer(src, np.uint8).copy()).cuda()
    out = torch.empty(int(gpu_ctx.L.hbam_bgzf_bound(len(src), 0)), dtype=torch.uint8, device="cuda")
    n = gpu_ctx.bgzf_compress(d, 0, out=out)
    comp = out[:n].cpu().numpy()
    rc, blocks = gpu_ctx.scan_blocks(comp)
    assert rc == 0
    ref = oracle_mod.scan_blocks(comp)
    for k in ("coff", "clen", "isize", "crc"):
        assert np.array_equal(blocks[k], ref[k])
    rc, u, off, st = gpu_ctx.inflate(comp, blocks, check_crc=True)
    assert rc == 0 and np.all(st == 0)
    assert u.tobytes() == src
    # ratio against zlib level 5 on the same stream (reported, loosely bounded)
    z = sum(len(zlib.compress(src[i:i + 65280], 5)) for i in range(0, len(src), 65280))
    assert n < 1.6 * z, (n, z)


# ---- GPU: the writer classes ----------------------------------------------------------------
@pytest.mark.gpu
def test_bam_record_writer_reads_back(gpu_ctx, oracle_mod, tmp_path):
    """BAMRecordWriter (header + every record of small_pe.bam via SAMRecordWritable) + the EOF
    block reads back through the oracle's BAMRecordReader to the same records."""
    from hadoop_bam.formats import SAMRecordWritable, BAMRecordBytes
    from hadoop_bam.output import BAMRecordWriter, EMPTY_GZIP_BLOCK, read_sam_header
    data = np.fromfile(os.path.join(GOLDEN, "small_pe.bam"), np.uint8)
    h = oracle_mod.read_header(data)
    ref = oracle_mod.read_split(data, h["first_voffset"], (len(data) << 16) | 0xffff)
    pay, off = oracle_mod.record_payloads(ref)
    header = read_sam_header(data, gpu_ctx)
    path = str(tmp_path / "out.bam")
    w = BAMRecordWriter(path, header, True, gpu_ctx)
    v = SAMRecordWritable()
    for i in range(ref["n"]):
        v.set(BAMRecordBytes(pay[int(off[i]):int(off[i + 1])].tobytes()))
        w.write(None, v)
    w.close()
    with open(path, "ab") as f:
        f.write(EMPTY_GZIP_BLOCK)
    out = np.fromfile(path, np.uint8)
    h2 = oracle_mod.read_header(out)
    assert h2["n_ref"] == h["n_ref"] and h2["l_text"] == h["l_text"]
    got = oracle_mod.read_split(out, h2["first_voffset"], (len(out) << 16) | 0xffff)
    assert got["n"] == ref["n"] and got["status"] == 0
    p2, _ = oracle_mod.record_payloads(got)
    assert p2.tobytes() == pay.tobytes()
    for k in ("key", "ref_id", "pos", "flag"):
        assert np.array_equal(got[k], ref[k])


@pytest.mark.gpu
def test_sort_output_merge_is_the_sorted_bam(gpu_ctx, oracle_mod, tmp_path):
    """The Sort plugin's output path: device decode + sort of two FileVirtualSplits, each
    rank's sorted records written as a header-less part by KeyIgnoringBAMOutputFormat from the
    device payload, mergeSAMInto (coordinate-sorted header, parts, EOF block): the merged BAM
    reads back to the oracle's total order."""
    import torch
    from hadoop_bam import sort
    from hadoop_bam.output import KeyIgnoringBAMOutputFormat, get_mergeable_work_file, merge_sam_into, read_sam_header
    data = np.fromfile(os.path.join(GOLDEN, "edge_unsorted_l1.bam"), np.uint8)
    h = oracle_mod.read_header(data)
    b, e = oracle_mod.file_splits(len(data), (len(data) + 1) // 2)
    vs, ve = oracle_mod.probabilistic_splits(data, b, e)
    ops = sort.HipSortOps(gpu_ctx)
    d = torch.from_numpy(data).cuda()
    keys, pays = [], []
    for a, z in zip(vs, ve):
        ref = oracle_mod.read_split(data, int(a), int(z))
        p, o = oracle_mod.record_payloads(ref)
        order = np.argsort(ref["key"], kind="stable")
        keys.append(ref["key"][order])
        pays += [p[int(o[i]):int(o[i + 1])].tobytes() for i in order]
    # the reduce side's total order over both splits' records (stable by split order)
    allk = np.concatenate(keys)
    want = [pays[i] for i in np.argsort(allk, kind="stable")]
    header = read_sam_header(data, gpu_ctx)
    header.setSortOrder("coordinate")
    fmt = KeyIgnoringBAMOutputFormat()
    fmt.setSAMHeader(header)
    fmt.setWriteHeader(False)
    wrk = tmp_path / "wrk"
    wrk.mkdir()
    runs = []
    for a, z in zip(vs, ve):
        rc, dc = gpu_ctx.decode_split_device(d, int(a), int(z), h["n_ref"])
        assert rc == 0 and dc.status == 0
        runs.append(ops.run_from_columns(dc))
    # one reducer: both map outputs merged by key (what the shuffle + reduce do)
    merged = ops.sort_received(torch.cat([r.keys for r in runs]), torch.cat([r.voffset for r in runs]),
                               torch.cat([r.block_size for r in runs]), torch.cat([r.payload for r in runs]))
    w = fmt.getRecordWriter(get_mergeable_work_file(str(wrk), "", "", "sort", 0), gpu_ctx)
    w.write_device(merged.payload, int(merged.offsets[-1].item()))
    w.close()
    out = str(tmp_path / "sorted.bam")
    merge_sam_into(out, str(wrk), "", "", header, work_filename="sort", ctx=gpu_ctx)
    assert os.listdir(str(wrk)) == []
    o = np.fromfile(out, np.uint8)
    h2 = oracle_mod.read_header(o)
    got = oracle_mod.read_split(o, h2["first_voffset"], (len(o) << 16) | 0xffff)
    assert got["status"] == 0 and got["n"] == len(want)
    p2, o2 = oracle_mod.record_payloads(got)
    assert [p2[int(o2[i]):int(o2[i + 1])].tobytes() for i in range(got["n"])] == want
    assert bytes(o[-28:]) == bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
