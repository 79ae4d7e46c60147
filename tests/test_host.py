"""Host-side mirror of the reference API (no GPU): FileVirtualSplit, Hadoop split sizing,
getKey0, SplittingBAMIndex, AnySAMInputFormat dispatch."""
import io
import os
import struct

import numpy as np

from conftest import GOLDEN


def test_file_virtual_split_length_and_writable():
    from hadoop_bam import FileVirtualSplit
    s = FileVirtualSplit("/data/x.bam", (100 << 16) | 5, (100 << 16) | 900, ["h1"])
    assert s.getLength() == 895  # same block: exact (FileVirtualSplit.java:64-69)
    s2 = FileVirtualSplit("/data/x.bam", (100 << 16) | 5, (300 << 16) | 1, [])
    assert s2.getLength() == (200 << 16)
    buf = io.BytesIO()
    s2.write(buf)
    raw = buf.getvalue()
    assert raw[0] == len("/data/x.bam") and raw[1:12] == b"/data/x.bam"
    assert struct.unpack(">qq", raw[12:]) == ((100 << 16) | 5, (300 << 16) | 1)
    t = FileVirtualSplit()
    t.readFields(io.BytesIO(raw))
    assert t == s2


def test_compute_file_splits_matches_oracle(oracle_mod):
    from hadoop_bam import compute_file_splits
    for flen, ss in [(1000, 100), (1050, 100), (1010, 100), (12345678, 1 << 20), (5, 100)]:
        b, e = oracle_mod.file_splits(flen, ss)
        got = compute_file_splits("f", flen, ss)
        assert [(x.getStart(), x.getStart() + x.getLength()) for x in got] == \
            [(int(x), int(y)) for x, y in zip(b, e)]


def test_get_key0_sign_extension():
    from hadoop_bam import BAMRecordReader
    assert BAMRecordReader.getKey0(3, 100) == (3 << 32) | 100
    assert BAMRecordReader.getKey0(3, -1) == -1
    assert BAMRecordReader.getKey(3, 101) == (3 << 32) | 100
    assert BAMRecordReader.getKey0(0x7fffffff, -5) == -5


def test_splitting_bam_index(oracle_mod, small_bam, tmp_path):
    from hadoop_bam import SplittingBAMIndex
    offs = oracle_mod.splitting_index(small_bam, granularity=1024)
    assert offs[-1] == len(small_bam) << 16
    raw = b"".join(struct.pack(">q", int(x)) for x in offs)
    idx = SplittingBAMIndex(io.BytesIO(raw))
    assert idx.size() == len(offs)
    mid = int(offs[5]) >> 16
    want = min(int(x) for x in offs if int(x) > (mid << 16))  # TreeSet.higher(mid << 16)
    assert idx.nextAlignment(mid) == want
    assert idx.prevAlignment(len(small_bam)) == len(small_bam) << 16


def test_any_sam_input_format_dispatch(tmp_path):
    from hadoop_bam import AnySAMInputFormat, Configuration
    p = tmp_path / "reads.dat"
    p.write_bytes(b"\x1f\x8b\x08\x04rest")
    assert AnySAMInputFormat().getFormat(str(p)) == "BAM"
    q = tmp_path / "reads.txt"
    q.write_bytes(b"@HD\tVN:1.6\n")
    assert AnySAMInputFormat().getFormat(str(q)) == "SAM"
    r = tmp_path / "lying.bam"
    r.write_bytes(b"@HD\n")
    assert AnySAMInputFormat().getFormat(str(r)) == "BAM"
    assert AnySAMInputFormat().getFormat(str(r), Configuration({
        "hadoopbam.anysam.trust-exts": "false"})) == "SAM"
