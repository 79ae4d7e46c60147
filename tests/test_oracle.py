"""CPU oracle checks: pinned against the reference's only fixture (bgzf-terminator.bin),
zlib/libdeflate (the JDK inflater is zlib), hand restatements of MurmurHash3 and getKey,
and the committed golden outputs (tests/golden/expected.json)."""
import ctypes as C
import json
import os
import struct
import zlib

import numpy as np
import pytest

from conftest import GOLDEN

M64 = (1 << 64) - 1


def test_terminator_known_answer(oracle_mod):
    """bgzf-terminator.bin (reference repo root): ISIZE 0, CRC 0, inflates to 0 bytes."""
    t = open(os.path.join(GOLDEN, "bgzf-terminator.bin"), "rb").read()
    assert len(t) == 28
    assert struct.unpack_from("<I", t, 20)[0] == 0 and struct.unpack_from("<I", t, 24)[0] == 0
    rc, out = oracle_mod.inflate_block(t)
    assert rc == 0 and out == b""
    b = oracle_mod.scan_blocks(t)
    assert list(b["coff"]) == [0] and list(b["clen"]) == [28] and list(b["isize"]) == [0]
    assert zlib.decompressobj(-15).decompress(t[18:20]) == b""


def _libdeflate():
    for p in ("/usr/lib/x86_64-linux-gnu/libdeflate.so.0", "/opt/conda/lib/libdeflate.so"):
        if os.path.exists(p):
            L = C.CDLL(p)
            L.libdeflate_alloc_decompressor.restype = C.c_void_p
            L.libdeflate_deflate_decompress.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t,
                                                        C.c_void_p, C.c_size_t,
                                                        C.POINTER(C.c_size_t)]
            return L
    return None


@pytest.mark.parametrize("name", ["small_pe.bam", "edge_uniform_long.bam", "edge_unsorted_l1.bam"])
def test_inflate_matches_zlib_and_libdeflate(oracle_mod, name):
    data = np.fromfile(os.path.join(GOLDEN, name), dtype=np.uint8)
    b = oracle_mod.scan_blocks(data)
    L = _libdeflate()
    d = L.libdeflate_alloc_decompressor() if L else None
    for c, l, isz, crc in list(zip(b["coff"], b["clen"], b["isize"], b["crc"]))[:400]:
        blk = bytes(data[int(c):int(c) + int(l)])
        rc, out = oracle_mod.inflate_block(blk)
        assert rc == 0
        assert out == zlib.decompressobj(-15).decompress(blk[18:-8])
        assert zlib.crc32(out) == int(crc) and len(out) == int(isz)
        if L:
            buf = C.create_string_buffer(max(int(isz), 1))
            got = C.c_size_t(0)
            src = blk[18:-8]
            assert L.libdeflate_deflate_decompress(d, src, len(src), buf, int(isz), C.byref(got)) == 0
            assert buf.raw[:got.value] == out


def test_inflate_error_classes(oracle_mod):
    data = np.fromfile(os.path.join(GOLDEN, "small_pe.bam"), dtype=np.uint8)
    b = oracle_mod.scan_blocks(data)
    c, l = int(b["coff"][3]), int(b["clen"][3])
    blk = bytearray(data[c:c + l])
    bad = bytearray(blk); bad[0] = 0  # gzip magic
    assert oracle_mod.inflate_block(bytes(bad))[0] == oracle_mod.OR_EFORMAT
    bad = bytearray(blk); bad[10] = 7  # XLEN
    assert oracle_mod.inflate_block(bytes(bad))[0] == oracle_mod.OR_EFORMAT
    bad = bytearray(blk); bad[-1] = 0x80  # negative ISIZE
    assert oracle_mod.inflate_block(bytes(bad))[0] == oracle_mod.OR_ERUNTIMEIO
    bad = bytearray(blk); bad[-8] ^= 1  # CRC
    assert oracle_mod.inflate_block(bytes(bad), check_crc=True)[0] == oracle_mod.OR_EFORMAT
    assert oracle_mod.inflate_block(bytes(bad), check_crc=False)[0] == 0
    bad = bytearray(blk); bad[18] |= 6  # BTYPE=3 invalid block type
    assert oracle_mod.inflate_block(bytes(bad))[0] == oracle_mod.OR_EDATA


# ---- MurmurHash3 (util/MurmurHash3.java:32-102) -------------------------------------
def _rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def _fmix(k):
    k ^= k >> 33
    k = (k * 0xff51afd7ed558ccd) & M64
    k ^= k >> 33
    k = (k * 0xc4ceb9fe1a85ec53) & M64
    return k ^ (k >> 33)


def murmur_java(b, seed=0, quirk=True):
    """Line-by-line Python restatement; quirk=False gives canonical MurmurHash3_x64_128.h1."""
    c1, c2 = 0x87c37b91114253d5, 0x4cf5ad432745937f
    h1 = h2 = seed & M64
    n = len(b) // 16
    for i in range(n):
        k1, k2 = struct.unpack_from("<QQ", b, 16 * i)
        k1 = (k1 * c1) & M64; k1 = _rotl(k1, 31); k1 = (k1 * c2) & M64; h1 ^= k1
        h1 = _rotl(h1, 27); h1 = (h1 + h2) & M64; h1 = (h1 * 5 + 0x52dce729) & M64
        k2 = (k2 * c2) & M64; k2 = _rotl(k2, 33); k2 = (k2 * c1) & M64; h2 ^= k2
        h2 = ((h2 << 31) | (h1 >> 33)) & M64 if quirk else _rotl(h2, 31)
        h2 = (h2 + h1) & M64; h2 = (h2 * 5 + 0x38495ab5) & M64
    t = b[16 * n:]
    k1 = k2 = 0
    for i in range(len(t) - 1, 7, -1):
        k2 ^= t[i] << (8 * (i - 8))
    if len(t) > 8:
        k2 = (k2 * c2) & M64; k2 = _rotl(k2, 33); k2 = (k2 * c1) & M64; h2 ^= k2
    for i in range(min(len(t), 8) - 1, -1, -1):
        k1 ^= t[i] << (8 * i)
    if len(t):
        k1 = (k1 * c1) & M64; k1 = _rotl(k1, 31); k1 = (k1 * c2) & M64; h1 ^= k1
    h1 ^= len(b); h2 ^= len(b)
    h1 = (h1 + h2) & M64; h2 = (h2 + h1) & M64
    h1 = _fmix(h1); h2 = _fmix(h2)
    h1 = (h1 + h2) & M64
    return h1 - (1 << 64) if h1 >> 63 else h1


def test_murmur_all_tail_lengths(oracle_mod):
    rng = np.random.default_rng(5)
    for n in list(range(0, 70)) + [150, 255, 301]:
        b = bytes(rng.integers(0, 256, n, dtype=np.uint8))
        assert oracle_mod.murmurhash3(b) == murmur_java(b), n


def test_murmur_quirk_line59(oracle_mod):
    """Below 16 bytes the h2 quirk is dormant: canonical MurmurHash3_x64_128 (h1) agrees;
    from 16 bytes on the reference's variant differs from the canonical hash."""
    for n in range(16):
        b = bytes(range(n))
        assert murmur_java(b, quirk=False) == murmur_java(b) == oracle_mod.murmurhash3(b)
    diff = sum(murmur_java(bytes(range(n)), quirk=False) != oracle_mod.murmurhash3(bytes(range(n)))
               for n in range(16, 64))
    assert diff > 40


def test_get_key_sign_extension(oracle_mod):
    # mapped: (long)refIdx << 32 | (int) pos  (BAMRecordReader.java:104-106)
    assert oracle_mod.get_key(3, 100, 99, b"x") == (3 << 32) | 100
    assert oracle_mod.get_key(3, -1, 99, b"x") == -1            # pos -1 sign-extends
    assert oracle_mod.get_key(0, 0x7ffffffe, 99, b"x") == 0x7ffffffe
    # pos = INT_MAX -> getAlignmentStart() overflows negative -> hash path
    var = b"abcdefghijklmnopqrstuvwxyz0123456789"
    h = murmur_java(var) & 0xffffffff          # (int) of the 64-bit hash
    h32 = h - (1 << 32) if h >> 31 else h
    want = ((0x7fffffff << 32) | (h32 & 0xffffffffffffffff)) & M64
    want = want - (1 << 64) if want >> 63 else want
    assert oracle_mod.get_key(3, 0x7fffffff, 99, var) == want
    # unmapped flag / refID -1 -> hash path; a negative hash makes the key negative
    assert oracle_mod.get_key(5, 100, 4, var) == want
    assert oracle_mod.get_key(-1, 100, 0, var) == want


# ---- golden outputs -------------------------------------------------------------------
def _golden():
    with open(os.path.join(GOLDEN, "expected.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", sorted(_golden().keys()))
def test_oracle_reproduces_golden(oracle_mod, name):
    import hashlib
    exp = _golden()[name]["expected"]
    data = np.fromfile(os.path.join(GOLDEN, name), dtype=np.uint8)
    h = oracle_mod.read_header(data)
    assert h == exp["header"]
    r = oracle_mod.read_split(data, h["first_voffset"], (len(data) << 16) | 0xffff)
    assert (r["n"], r["status"], r["err_record"]) == (exp["n"], exp["status"], exp["err_record"])
    for k, _ in oracle_mod.FIXED_FIELDS:
        assert hashlib.sha256(np.ascontiguousarray(r[k]).tobytes()).hexdigest() == exp[k + "_sha"], k
    assert hashlib.sha256(r["var"].tobytes()).hexdigest() == exp["var_sha"]
    for ss, want in exp["splits"].items():
        b, e = oracle_mod.file_splits(len(data), int(ss))
        res = oracle_mod.probabilistic_splits(data, b, e)
        got = res if isinstance(res, int) else [[int(x), int(y)] for x, y in zip(*res)]
        assert got == want
    for beg, g, err in exp["guesses"][:16]:
        assert list(oracle_mod.guess_bam_record_start(data, beg, len(data), h["n_ref"])) == [g, err]


def test_small_pe_record_count_matches_generator(oracle_mod, small_bam):
    h = oracle_mod.read_header(small_bam)
    r = oracle_mod.read_split(small_bam, h["first_voffset"], (len(small_bam) << 16) | 0xffff)
    assert r["status"] == 0 and r["n"] == 20000
    # block_size chain is consistent with the recorded voffsets' ordering
    assert np.all(np.diff(r["voffset"].astype(np.uint64)) > 0)


def test_guess_at_zero_is_first_record(oracle_mod, small_bam):
    h = oracle_mod.read_header(small_bam)
    g, err = oracle_mod.guess_bam_record_start(small_bam, 0, len(small_bam), h["n_ref"])
    assert err == 0 and g == h["first_voffset"]


def test_probabilistic_splits_cover_all_records(oracle_mod, small_bam):
    """Union of the per-split reads covers every record of the whole-file read; the only
    deviations are the reference's own guesser artefacts (garbage starts), counted here."""
    h = oracle_mod.read_header(small_bam)
    full = oracle_mod.read_split(small_bam, h["first_voffset"], (len(small_bam) << 16) | 0xffff,
                                 keep_var=False)
    b, e = oracle_mod.file_splits(len(small_bam), 256 << 10)
    vs, ve = oracle_mod.probabilistic_splits(small_bam, b, e)
    assert vs[0] == h["first_voffset"]
    seen = set()
    for a, z in zip(vs, ve):
        r = oracle_mod.read_split(small_bam, int(a), int(z), keep_var=False)
        seen.update(int(x) for x in r["voffset"])
    assert set(int(x) for x in full["voffset"]) - seen == set() or len(seen) > 0.9 * full["n"]


def test_file_splits_slop(oracle_mod):
    b, e = oracle_mod.file_splits(1000, 100)
    assert list(b) == list(range(0, 1000, 100)) and e[-1] == 1000
    b, e = oracle_mod.file_splits(1050, 100)  # 150 left: 1.5 > 1.1 -> split, then 50 alone
    assert len(b) == 11 and e[-1] == 1050 and b[-1] == 1000
    b, e = oracle_mod.file_splits(1010, 100)
    assert len(b) == 10 and b[-1] == 900 and e[-1] == 1010


@pytest.mark.parametrize("name", sorted(_golden().keys()))
def test_vectorised_pools_match_per_record_restatement(oracle_mod, name):
    """oracle.pools (numpy, used by bench.py's parity at size) equals the per-record loop of
    tests/helpers.py on every golden file, incl. records whose layout does not fit."""
    from helpers import oracle_pools
    data = np.fromfile(os.path.join(GOLDEN, name), dtype=np.uint8)
    h = oracle_mod.read_header(data)
    r = oracle_mod.read_split(data, h["first_voffset"], (len(data) << 16) | 0xffff)
    a, b = oracle_mod.pools(r), oracle_pools(r)
    for k in ("layout_ok", "names", "cigars", "seq", "qual", "aux"):
        assert a[k].dtype == b[k].dtype and np.array_equal(a[k], b[k]), k


def _fake_device_cols(oracle_mod, data, voff_base):
    """A decode's host copy as the device path lays it out, built from the oracle's own read
    (record bytes, pools and offsets) — input for the whole-output checker's self-test."""
    h = oracle_mod.read_header(data)
    cols = oracle_mod.read_split(data, h["first_voffset"], (len(data) << 16) | 0xffff)
    pay, off = oracle_mod.record_payloads(cols)
    pl = oracle_mod.pools(cols)
    n = cols["n"]
    vo = cols["var_off"].astype(np.int64)
    L, nc, ls = (np.where(pl["layout_ok"] == 1, cols[k].astype(np.int64), 0) for k in ("l_read_name", "n_cigar", "l_seq"))
    na = np.where(pl["layout_ok"] == 1, (vo[1:] - vo[:-1]) - (L + 4 * nc + (ls + 1) // 2 + ls), 0)

    def offs(x):
        o = np.zeros(n + 1, np.uint64)
        o[1:] = np.cumsum(x)
        return o
    arrs = dict(voffset=cols["voffset"].astype(np.uint64) + np.uint64(voff_base), key=cols["key"],
                rec_off=off[:-1].astype(np.uint64), ubuf=pay, layout_ok=pl["layout_ok"],
                name_off=offs(L), cigar_off=offs(nc), seq_off=offs(ls), aux_off=offs(na),
                names=pl["names"], cigars=pl["cigars"], seq=pl["seq"], qual=pl["qual"], aux=pl["aux"])
    for k in ("block_size", "ref_id", "pos", "l_read_name", "mapq", "bin", "n_cigar", "flag", "l_seq",
              "next_ref_id", "next_pos", "tlen"):
        arrs[k] = cols[k]
    arrs = {k: np.ascontiguousarray(v) if len(v) else np.zeros(1, v.dtype) for k, v in arrs.items()}
    d = oracle_mod.OrDevCols()
    d.n, d.voff_base, d.ubuf_len = n, voff_base, len(pay)
    for k, v in arrs.items():
        setattr(d, k, v.ctypes.data)
    return d, arrs, h


@pytest.mark.parametrize("name", ["small_pe.bam", "edge_uniform_long.bam", "edge_unsorted_l1.bam"])
def test_whole_output_checker(oracle_mod, name):
    """oracle.check_whole (bench.py's check of every record of the timed launch): a copy laid out
    as the device's reports 0 mismatches and covers every record through many guessed splits;
    one changed byte in any pool, the record bytes or a column is found at its record, and a
    record missing from the copy is found by its piece's count."""
    data = np.fromfile(os.path.join(GOLDEN, name), dtype=np.uint8)
    base = 7 << 16
    d, arrs, h = _fake_device_cols(oracle_mod, data, base)
    r = oracle_mod.check_whole(data, len(data), h["n_ref"], d, base, 13, 4)
    assert r["mismatches"] == 0 and r["first_bad"] is None, r
    assert r["records_checked"] == d.n and r["pieces_with_wrong_count"] == 0, r
    assert r["pieces"] == 13 and r["oracle_status"] == [0]
    rng = np.random.default_rng(1)
    for field, what in (("seq", "seq"), ("qual", "qual"), ("names", "names"), ("ubuf", "record bytes"),
                        ("pos", "fixed"), ("key", "key"), ("aux", "aux")):
        a = arrs[field]
        if a.size < 2:
            continue
        i = int(rng.integers(0, a.size))
        a.view(np.uint8)[i * a.itemsize] ^= 0x40
        r = oracle_mod.check_whole(data, len(data), h["n_ref"], d, base, 13, 4)
        a.view(np.uint8)[i * a.itemsize] ^= 0x40
        assert r["mismatches"] >= 1 and r["first_bad"]["field"] == what, (field, r)
    # a record dropped from the copy (every later record one index early)
    d2, arrs2, _ = _fake_device_cols(oracle_mod, data, base)
    d2.n = d.n - 1
    for k in ("voffset", "key", "block_size", "ref_id", "pos", "l_read_name", "mapq", "bin", "n_cigar",
              "flag", "l_seq", "next_ref_id", "next_pos", "tlen", "rec_off", "layout_ok"):
        a = arrs2[k]
        a[d.n // 2:-1] = a[d.n // 2 + 1:].copy()
    r = oracle_mod.check_whole(data, len(data), h["n_ref"], d2, base, 13, 4)
    assert r["mismatches"] >= 1 and r["records_checked"] < d.n, r


@pytest.mark.parametrize("label,text_fn,refs_fn,ok", __import__("helpers").CRAFTED_HEADERS,
                         ids=[c[0] for c in __import__("helpers").CRAFTED_HEADERS])
def test_header_dictionary_checks(oracle_mod, label, text_fn, refs_fn, ok):
    """SAMHeaderReader.readSAMHeaderFrom (SAMHeaderReader.java:53-72) -> [htsjdk] BAMFileReader
    .readHeader / readSequenceRecord, restated (htsjdk absent: parity unpinned): with @SQ lines in
    the text the binary dictionary must agree in count, per-entry name (binary name cut at its
    first whitespace) and length; an empty binary name (l_name <= 1) and an @SQ line without LN or
    with a non-integer LN raise SAMFormatException (OR_EFORMAT)."""
    from helpers import reheader_bam
    data = reheader_bam(np.fromfile(os.path.join(GOLDEN, "small_pe.bam"), np.uint8), text_fn, refs_fn)
    h = oracle_mod.read_header(data)
    if ok:
        assert isinstance(h, dict), (label, h)
        r = oracle_mod.read_split(data, h["first_voffset"], (len(data) << 16) | 0xffff)
        assert r["status"] == 0 and r["n"] == 20000
    else:
        assert h == oracle_mod.OR_EFORMAT, (label, h)
