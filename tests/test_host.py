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


def test_generate_range_concatenates_to_one_file(genbam, oracle_mod):
    """Byte ranges of one synthetic file (bench.py --gpus N: one range per rank) concatenate
    to the whole file, which the oracle reads with the generator's record count."""
    kw = dict(seed=9, segment=400, threads=4)
    whole = genbam.generate_range(6, 0, 6, header=True, tail=True, **kw)
    parts = [genbam.generate_range(6, 0, 2, header=True, **kw), genbam.generate_range(6, 2, 3, **kw),
             genbam.generate_range(6, 5, 1, tail=True, **kw)]
    assert np.array_equal(np.concatenate(parts), whole)
    assert sum(p.n_records for p in parts) == whole.n_records
    h = oracle_mod.read_header(whole)
    r = oracle_mod.read_split(whole, h["first_voffset"], (len(whole) << 16) | 0xffff)
    assert r["status"] == 0 and r["n"] == whole.n_records


def test_host_murmurhash3_matches_oracle(oracle_mod):
    """formats.murmurhash3_bytes (the host getKey(SAMRecord) hash) equals the oracle's
    MurmurHash3.murmurhash3(byte[], seed) for every tail length and negative seeds."""
    from hadoop_bam.formats import murmurhash3_bytes
    rng = np.random.default_rng(5)
    for n in list(range(0, 40)) + [255, 1000]:
        b = rng.integers(0, 256, n).astype(np.uint8).tobytes()
        for seed in (0, 7, -3):
            assert murmurhash3_bytes(b, seed) == oracle_mod.murmurhash3(b, seed), (n, seed)


def test_record_bytes_fields_and_static_get_key(oracle_mod):
    """SAMRecordWritable.readFields -> lazy record over the wire bytes: its fixed fields equal
    the oracle's decode, and the static BAMRecordReader.getKey(SAMRecord) (Sort.java:292) equals
    the key the reader emits, unmapped-hash keys included."""
    from hadoop_bam import BAMRecordReader, SAMRecordWritable
    data = np.fromfile(os.path.join(GOLDEN, "small_pe.bam"), dtype=np.uint8)
    h = oracle_mod.read_header(data)
    cols = oracle_mod.read_split(data, h["first_voffset"], (len(data) << 16) | 0xffff)
    pay, off = oracle_mod.record_payloads(cols)
    n_hash = 0
    for i in range(0, cols["n"], 7):
        w = SAMRecordWritable()
        w.readFields(io.BytesIO(pay[off[i]:off[i + 1]].tobytes()))
        r = w.get()
        assert r.getReferenceIndex() == cols["ref_id"][i]
        assert r.getAlignmentStart() == int(np.int32(cols["pos"][i]) + np.int32(1))
        assert r.getFlags() == cols["flag"][i]
        assert BAMRecordReader.getKey(r) == int(cols["key"][i])
        n_hash += int(cols["key"][i] >> 32 == 0x7fffffff or cols["key"][i] < 0)
        out = io.BytesIO()
        w.write(out)
        assert out.getvalue() == pay[off[i]:off[i + 1]].tobytes()
    assert n_hash > 0
