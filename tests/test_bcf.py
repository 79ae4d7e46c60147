"""BCF over the BGZF layer: BCFSplitGuesser, BCFRecordReader and the BCF half
of VCFInputFormat on the device against the CPU restatement (oracle/hbam_oracle_bcf.c).

Parity: the candidate scan (BCFSplitGuesser.guessNextBCFPos), the BGZF positioning and the
stream plumbing (PositionalBufferedStream fills, BGZFLimitingStream) are the reference's own
code; the record decode is a restated subset of htsjdk's BCF2Codec (absent here) — parity
unpinned beyond the self-generated files below (tests/bcf_records.py writes BCF2.1 per spec)."""
import numpy as np
import pytest

import bcf_records
from helpers import bgzf_pack

SAMPLES60 = tuple("S%d" % i for i in range(60))


def _record_starts(u, header_len):
    p, out = header_len, []
    while p + 8 <= len(u):
        out.append(p)
        p += 8 + int.from_bytes(u[p:p + 4], "little") + int.from_bytes(u[p + 4:p + 8], "little")
    return out


@pytest.fixture(scope="module")
def bcf_files():
    """plain: uncompressed BCF; bgzf: the same stream in BGZF (population-like, ~6x);
    bgzf_low: a poorly compressible BGZF BCF (every guess window ends in a truncated block);
    bad_*: corruptions."""
    plain = bcf_records.bcf_stream(6000, seed=3, samples=SAMPLES60, hom_ref=0.97)
    low = bcf_records.bcf_stream(8000, seed=4)
    f = {"plain": plain, "bgzf": bgzf_pack(plain), "bgzf_low": bgzf_pack(low)}
    import oracle
    h = oracle.bcf_header(plain)
    st = _record_starts(plain, h["header_len"])
    b = bytearray(plain)
    r = st[2500]
    b[r + 8:r + 12] = (99).to_bytes(4, "little")  # CHROM outside the dictionary
    f["bad_contig"] = bytes(b)
    b = bytearray(plain)
    r = st[4000]
    b[r:r + 4] = (0xfffffff0).to_bytes(4, "little")  # negative l_shared
    f["bad_size"] = bytes(b)
    b = bytearray(plain)
    r = st[3100]
    b[r + 28] ^= 0x01  # sample count: TribbleException
    f["bad_samples"] = bytes(b)
    f["trunc_plain"] = plain[:st[5000] + 21]
    z = bgzf_pack(plain)
    f["trunc_bgzf"] = z[:len(z) - 28 - 1000]  # the last data block cut short
    # a corrupt DEFLATE stream in a middle block: the reader's fill that reaches it throws
    zb = bytearray(z)
    p, k = 0, 0
    while True:
        bl = int.from_bytes(zb[p + 16:p + 18], "little") + 1
        if k == 12:
            for j in range(p + 18, p + 40):
                zb[j] ^= 0x5a
            break
        p += bl
        k += 1
    f["bad_block"] = bytes(zb)
    return f


@pytest.fixture(scope="module")
def headers(bcf_files):
    import oracle
    return {k: oracle.bcf_header(v) for k, v in bcf_files.items()}


# ---- the restatement itself (CPU) ------------------------------------------------------------------
def test_oracle_header_and_records(bcf_files, headers):
    import oracle
    h = headers["plain"]
    assert (h["n_contig"], h["n_sample"], h["n_dict"], h["bgzf"]) == (25, 60, 6, False)
    assert headers["bgzf"]["bgzf"] and headers["bgzf"]["header_len"] == h["header_len"]
    r = oracle.read_bcf_split(bcf_files["plain"], 0, len(bcf_files["plain"]), h)
    assert r["n"] == 6000 and r["status"] == 0
    assert list(r["rel"]) == _record_starts(bcf_files["plain"], h["header_len"])
    assert np.array_equal(r["key"], (r["chrom"].astype(np.int64) << 32) | r["pos"].astype(np.int64))


def test_oracle_uncompressed_splits_partition_the_records(bcf_files, headers):
    import oracle
    data, h = bcf_files["plain"], headers["plain"]
    keys = []
    for a, ln in oracle.bcf_splits(data, 200000, h):
        r = oracle.read_bcf_split(data, a, ln, h)
        assert r["status"] == 0
        keys.append(r["key"])
    whole = oracle.read_bcf_split(data, 0, len(data), h)
    assert np.array_equal(np.concatenate(keys), whole["key"])


def test_oracle_bgzf_guesses_land_on_records(bcf_files, headers):
    import oracle
    z, h = bcf_files["bgzf"], headers["bgzf"]
    sc = oracle.scan_blocks(z)
    coff = list(sc["coff"])
    uo = np.concatenate([[0], np.cumsum(sc["isize"])])
    starts = set(_record_starts(bcf_files["plain"], h["header_len"]))
    rng = np.random.default_rng(5)
    hits = 0
    for beg in rng.integers(0, len(z) - 1, 30):
        g, e = oracle.guess_bcf_record_start(z, int(beg), len(z), h)
        assert e == 0
        if g != len(z):
            hits += 1
            assert int(uo[coff.index(g >> 16)]) + (g & 0xffff) in starts
    assert hits >= 25


def test_oracle_bgzf_split_reads_to_the_end_of_file(bcf_files, headers):
    """BGZFLimitingStream stops only in a block starting exactly at the split end
    (BCFRecordReader.java:206), so a BGZF split reads every record after its start."""
    import oracle
    z, h = bcf_files["bgzf"], headers["bgzf"]
    sp = oracle.bcf_splits(z, 100000, h)
    assert len(sp) >= 2
    r0 = oracle.read_bcf_split(z, sp[0][0], sp[0][1], h)
    assert r0["n"] == 6000 and r0["status"] == 0
    r1 = oracle.read_bcf_split(z, sp[1][0], sp[1][1], h)
    assert 0 < r1["n"] < 6000 and r1["status"] == 0


# ---- device vs restatement -------------------------------------------------------------------------
NAMES = ["plain", "bgzf", "bgzf_low", "bad_contig", "bad_size", "bad_samples", "trunc_plain", "trunc_bgzf",
         "bad_block"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["plain", "bgzf", "bgzf_low"])
def test_header_matches_oracle(gpu_ctx, bcf_files, headers, name):
    h = gpu_ctx.bcf_parse_header(bcf_files[name][:1 << 20])
    o = headers[name]
    assert isinstance(h, dict), h
    for k in ("n_contig", "n_sample", "n_dict", "header_len", "bgzf"):
        assert h[k] == o[k], k


def _windows(ctx, data, beg, end, bgzf):
    wl = [ctx.guess_bcf_window_len(len(data), b, e, bgzf) for b, e in zip(beg, end)]
    off = np.zeros(len(beg) + 1, np.uint64)
    off[1:] = np.cumsum(wl)
    w = b"".join(bytes(data[int(b):int(b) + n]) for b, n in zip(beg, wl))
    return w, off


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_guesses_match_oracle(gpu_ctx, bcf_files, headers, name):
    import oracle
    data, h = bcf_files[name], headers[name]
    rng = np.random.default_rng(11)
    n = len(data)
    beg = np.concatenate([[0, 1, 100, h["header_len"] - 3, n - 40, n - 5000, n - 70000],
                          rng.integers(0, n, 40)]).clip(0, n - 1).astype(np.int64)
    end = np.minimum(beg + np.where(np.arange(len(beg)) % 3 == 0, 1 << 27, 150000), n).astype(np.int64)
    w, off = _windows(gpu_ctx, data, beg, end, h["bgzf"])
    rc, out, err = gpu_ctx.guess_bcf_windows(w, off, n, beg, end, h)
    assert rc == 0, gpu_ctx.last_error()
    for i in range(len(beg)):
        g, e = oracle.guess_bcf_record_start(data, int(beg[i]), int(end[i]), h)
        assert (int(out[i]), int(err[i])) == (g, e), (i, int(beg[i]), int(end[i]))


@pytest.mark.gpu
@pytest.mark.parametrize("name,split_size", [("plain", 150000), ("plain", 700000), ("bgzf", 100000),
                                             ("bgzf", 40000)])
def test_splits_and_reads_match_oracle(gpu_ctx, bcf_files, headers, name, split_size):
    import oracle
    data, h = bcf_files[name], headers[name]
    sp = oracle.bcf_splits(data, split_size, h)
    assert isinstance(sp, list) and sp
    for a, b in sp:
        ref = oracle.read_bcf_split_ex(data, a, b, h)
        got = gpu_ctx.bcf_decode_split(data, h, a, b, keep_data=True)
        assert got["rc"] == 0, got
        assert (got["n"], got["status"]) == (ref["n"], ref["status"]), (a, b)
        # every column BCFRecordReader's records carry, and each record's bytes
        for k in ("rel", "chrom", "pos", "key", "l_shared", "l_indiv", "rlen", "qual", "n_allele_info",
                  "n_fmt_sample"):
            assert np.array_equal(got[k], ref[k]), k
        recs = b"".join(bytes(got["data"][int(o):int(o) + 8 + int(ls) + int(li)])
                        for o, ls, li in zip(got["rec_off"], got["l_shared"], got["l_indiv"]))
        assert recs == ref["bytes"]


def test_oracle_bcf_columns_consistent(bcf_files, headers):
    """read_bcf_split_ex agrees with read_bcf_split and its record bytes parse back to its columns."""
    import struct
    import oracle
    data, h = bcf_files["plain"], headers["plain"]
    a = oracle.read_bcf_split(data, 0, len(data), h)
    b = oracle.read_bcf_split_ex(data, 0, len(data), h)
    assert a["n"] == b["n"] == 6000
    for k in ("rel", "chrom", "pos", "key"):
        assert np.array_equal(a[k], b[k])
    for i in (0, 1, 2999, 5999):
        r = b["bytes"][int(b["boff"][i]):int(b["boff"][i + 1])]
        ls, li, chrom, pos, rlen, qual = struct.unpack_from("<iiiiiI", r, 0)
        assert (ls, li, chrom, pos, rlen, qual) == (b["l_shared"][i], b["l_indiv"][i], b["chrom"][i],
                                                    b["pos"][i], b["rlen"][i], b["qual"][i])
        assert len(r) == 8 + ls + li


@pytest.mark.gpu
def test_bcf_split_inflates_its_own_blocks(gpu_ctx, bcf_files, headers, tmp_path):
    """a BGZF split inflates only the blocks BGZFLimitingStream lets it read, not the
    rest of the file.  The stream stops in vEnd's block (BCFRecordReader.java:206-235).
    VCFInputFormat's BCF splits end at raw FileSplit ends (vEnd = end << 16 | 0xffff), which are
    never a block start, so those splits read -- and must inflate -- to the end of the file, as the
    reference does; the mirror's window still grows only while the decode asks for
    more.  A split whose vEnd lies in a block inflates at most up to the block after vEnd's."""
    import oracle
    from hadoop_bam import bcf
    data, h = bcf_files["bgzf"], headers["bgzf"]
    size = 60000
    sp = oracle.bcf_splits(data, size, h)
    assert len(sp) >= 4
    path = tmp_path / "b.bcf"
    path.write_bytes(data)
    splits = bcf.VCFInputFormat().getSplits(str(path), size)
    for s, (a, b) in zip(splits, sp):
        got = gpu_ctx.bcf_decode_split(data[a >> 16:], h, a, b, comp_base=a >> 16, file_len=len(data))
        ref = oracle.read_bcf_split(data, a, b, h)
        assert (got["n"], got["status"]) == (ref["n"], ref["status"])
        assert np.array_equal(got["key"], ref["key"])
        rr = bcf.VCFInputFormat().createRecordReader(s)
        keys, exc = bcf.record_keys(rr)
        assert exc is None and np.array_equal(keys, ref["key"])
        assert rr.window_bytes <= ((b >> 16) - (a >> 16)) + bcf.BCF_WINDOW_TAIL
    # FileVirtualSplits ending inside a block: the stream stops there (mid-record here, so the
    # decode ends with the TribbleException the oracle raises too), and the device inflates only
    # up to the block after vEnd's, although the whole rest of the file is handed in
    blk = oracle.scan_blocks(data)
    coff = [int(x) for x in blk["coff"]]
    cum = np.concatenate([[0], np.cumsum(np.asarray(blk["isize"], np.int64))])
    a = sp[1][0]
    s0 = coff.index(a >> 16)
    assert s0 + 8 < len(coff)
    for k in (s0 + 1, s0 + 3, s0 + 6):
        v_end = coff[k] << 16 | 100
        got = gpu_ctx.bcf_decode_split(data[a >> 16:], h, a, v_end, comp_base=a >> 16, file_len=len(data))
        ref = oracle.read_bcf_split(data, a, v_end, h)
        assert (got["n"], got["status"]) == (ref["n"], ref["status"])
        assert np.array_equal(got["key"], ref["key"])
        assert got["timing"]["ubuf_bytes"] <= cum[k + 2] - cum[s0], (k, got["timing"]["ubuf_bytes"])



@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES[3:])
def test_corrupt_files_raise_what_the_oracle_raises(gpu_ctx, bcf_files, headers, name):
    import oracle
    data, h = bcf_files[name], headers[name]
    start = h["header_len"] if not h["bgzf"] else 0
    if h["bgzf"]:
        import hadoop_bam.bcf  # noqa: F401
        start = gpu_ctx.bcf_parse_header(data[:1 << 20])["first_voffset"]
        stop = (len(data) << 16) | 0xffff
    else:
        stop = len(data) - start
    ref = oracle.read_bcf_split(data, start, stop, h)
    got = gpu_ctx.bcf_decode_split(data, h, start, stop)
    assert got["rc"] == 0, got
    assert ref["status"] != 0
    assert (got["n"], got["status"]) == (ref["n"], ref["status"])
    assert np.array_equal(got["key"], ref["key"])


@pytest.mark.gpu
def test_mirror_vcf_input_format(bcf_files, headers, tmp_path):
    """VCFInputFormat.getSplits + BCFRecordReader (the mirror) over a BGZF and a plain file."""
    import oracle
    from hadoop_bam import bcf
    for name, size in (("bgzf", 100000), ("plain", 300000)):
        path = tmp_path / (name + ".bcf")
        path.write_bytes(bcf_files[name])
        splits = bcf.VCFInputFormat().getSplits(str(path), size)
        ref = oracle.bcf_splits(bcf_files[name], size, headers[name])
        got = [(s.getStartVirtualOffset(), s.getEndVirtualOffset()) if name == "bgzf"
               else (s.getStart(), s.getLength()) for s in splits]
        assert got == [tuple(x) for x in ref]
        for s, (a, b) in zip(splits, ref):
            keys, exc = bcf.record_keys(bcf.VCFInputFormat().createRecordReader(s))
            r = oracle.read_bcf_split(bcf_files[name], a, b, headers[name])
            assert exc is None and np.array_equal(keys, r["key"])


def _alt_header_stream():
    """A BCF stream whose header carries ##ALT and ##contig lines between the dictionary lines."""
    import struct
    text = bcf_records.header_text().replace(
        "##FORMAT=<ID=GT", '##ALT=<ID=DEL,Description="Deletion">\n##ALT=<ID=DUP,Description="Dup">\n'
        "##FORMAT=<ID=GT").encode() + b"\0"
    return b"BCF\x02\x02" + struct.pack("<i", len(text)) + text


def test_dictionary_rule_with_alt_and_contig_lines():
    """The string dictionary restated as BCF2Utils.makeDictionary over FILTER / INFO / FORMAT IDs
    (PASS first, first occurrence): ##ALT and ##contig lines are not in it.  Whether htsjdk 1.131's
    shouldBeAddedToDictionary() also admits those VCFSimpleHeaderLine subclasses is unverified here
    (no htsjdk): parity unpinned, noted in include/hbam.h."""
    import oracle
    h = oracle.bcf_header(_alt_header_stream())
    assert h["n_dict"] == len(bcf_records.DICT) == 6
    assert h["n_contig"] == 25


@pytest.mark.gpu
def test_dictionary_rule_with_alt_and_contig_lines_on_device(gpu_ctx):
    import oracle
    b = _alt_header_stream()
    h = gpu_ctx.bcf_parse_header(b)
    o = oracle.bcf_header(b)
    assert isinstance(h, dict), h
    assert (h["n_dict"], h["n_contig"], h["header_len"]) == (o["n_dict"], o["n_contig"], o["header_len"]) == (6, 25, len(b))
