"""Test helpers: derive the columnar pools the GPU emits from the oracle's raw variable
blocks (name | cigar | packed seq | qual | aux), so both sides compare field by field."""
import numpy as np

SEQ_ALPHA = np.frombuffer(b"=ACMGRSVTWYHKDBN", dtype=np.uint8)

FIELDS = ("voffset", "key", "block_size", "ref_id", "pos", "l_read_name", "mapq", "bin",
          "n_cigar", "flag", "l_seq", "next_ref_id", "next_pos", "tlen")


def oracle_pools(ref):
    n = ref["n"]
    names, cig, seq, qual, aux = [], [], [], [], []
    layout = np.zeros(n, np.uint8)
    for i in range(n):
        v = ref["var"][int(ref["var_off"][i]):int(ref["var_off"][i + 1])]
        L = int(ref["l_read_name"][i])
        nc = int(ref["n_cigar"][i])
        ls = int(ref["l_seq"][i])
        fixed = L + 4 * nc + (ls + 1) // 2 + ls
        if ls < 0 or fixed > len(v):
            continue
        layout[i] = 1
        p = 0
        names.append(v[p:p + L]); p += L
        cig.append(v[p:p + 4 * nc].view(np.uint32) if nc else np.zeros(0, np.uint32)); p += 4 * nc
        packed = v[p:p + (ls + 1) // 2]; p += (ls + 1) // 2
        hi = packed >> 4
        lo = packed & 15
        codes = np.empty(2 * len(packed), np.uint8)
        codes[0::2] = hi
        codes[1::2] = lo
        seq.append(SEQ_ALPHA[codes[:ls]])
        qual.append(v[p:p + ls]); p += ls
        aux.append(v[p:])
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)
    return dict(layout_ok=layout, names=cat(names, np.uint8), cigars=cat(cig, np.uint32),
                seq=cat(seq, np.uint8), qual=cat(qual, np.uint8), aux=cat(aux, np.uint8))


def assert_same_split(got, ref, pools=True):
    assert got["n"] == ref["n"], (got["n"], ref["n"])
    assert got["status"] == ref["status"], (got["status"], ref["status"])
    if ref["status"] != 0:
        assert got["err_record"] == ref["err_record"]
    for k in FIELDS:
        assert np.array_equal(got[k], ref[k]), "column %s differs" % k
    if pools:
        op = oracle_pools(ref)
        assert np.array_equal(got["layout_ok"], op["layout_ok"])
        for k in ("names", "cigars", "seq", "qual", "aux"):
            assert np.array_equal(got[k], op[k]), "pool %s differs" % k


def bgzf_pack(u, level=5, block=65280):
    """BGZF members (zlib raw deflate) of the inflated stream u, plus the EOF block."""
    import struct
    import zlib
    out = []
    for p in range(0, len(u), block):
        chunk = bytes(u[p:p + block])
        co = zlib.compressobj(level, zlib.DEFLATED, -15)
        cd = co.compress(chunk) + co.flush()
        out.append(b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" +
                   struct.pack("<H", len(cd) + 25) + cd + struct.pack("<II", zlib.crc32(chunk), len(chunk)))
    out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    return b"".join(out)


def bam_stream(data):
    """inflated stream of a whole BAM (zlib)"""
    import struct
    import zlib
    d = bytes(data)
    u, p = [], 0
    while p + 18 <= len(d):
        bs = struct.unpack_from("<H", d, p + 16)[0] + 1
        u.append(zlib.decompressobj(-15).decompress(d[p + 18:p + bs - 8]))
        p += bs
    return b"".join(u)


def redictionary_bam(data, prepend=((b"chrNEW", 5000),), drop_last=1):
    """A second input with a different dictionary, built from a BAM's records: `prepend` new
    sequences, then the input's dictionary without its last `drop_last` sequences; every record
    kept, its refIDs shifted up by len(prepend) (records on the dropped sequences left out).
    Merged after the original (SamFileHeaderMerger.mergeSequences), the new sequences come first,
    so the ORIGINAL's indices move up by len(prepend) — beyond its own dictionary when that
    exceeds what it has after its records' sequences (the reference's IllegalArgumentException,
    see hbam_merge_remap) — and this file's indices stay."""
    import struct
    u = bam_stream(data)
    lt = struct.unpack_from("<i", u, 4)[0]
    text = u[8:8 + lt]
    p = 8 + lt
    n = struct.unpack_from("<i", u, p)[0]
    p += 4
    refs = []
    for _ in range(n):
        ln = struct.unpack_from("<i", u, p)[0]
        refs.append((u[p + 4:p + 3 + ln], struct.unpack_from("<i", u, p + 4 + ln)[0]))
        p += 8 + ln
    keep = len(refs) - drop_last
    new_refs = list(prepend) + refs[:keep]
    lines = [ln for ln in text.split(b"\n") if not ln.startswith(b"@SQ")]
    sq = [b"@SQ\tSN:" + nm + b"\tLN:" + str(ln).encode() for nm, ln in new_refs]
    hd = [ln for ln in lines if ln.startswith(b"@HD")]
    rest = [ln for ln in lines if ln and not ln.startswith(b"@HD")]
    new_text = b"\n".join(hd + sq + rest) + b"\n"
    out = [b"BAM\x01", struct.pack("<i", len(new_text)), new_text, struct.pack("<i", len(new_refs))]
    for nm, ln in new_refs:
        out += [struct.pack("<i", len(nm) + 1), nm, b"\0", struct.pack("<i", ln)]
    k = len(prepend)
    while p + 4 <= len(u):
        bs = struct.unpack_from("<i", u, p)[0]
        r = bytearray(u[p:p + 4 + bs])
        p += 4 + bs
        ref, mref = struct.unpack_from("<i", r, 4)[0], struct.unpack_from("<i", r, 24)[0]
        if ref >= keep or mref >= keep:
            continue
        if ref >= 0:
            struct.pack_into("<i", r, 4, ref + k)
        if mref >= 0:
            struct.pack_into("<i", r, 24, mref + k)
        out.append(bytes(r))
    return np.frombuffer(bgzf_pack(b"".join(out)), np.uint8).copy(), refs, new_refs


def regroup_bam(data, text_fn, rg_fn, ref_fn=None):
    """A copy of a BAM with its header text replaced by text_fn(text) and each record's first RG
    tag replaced by rg_fn(i, value): None drops the tag, bytes = a new Z value, (type, raw) any
    typed value (multi-input Sort group-collision tests); ref_fn(i, refID) -> the record's new
    refID (and mate refID, where placed)."""
    import struct
    import oracle
    u = bam_stream(data)
    lt = struct.unpack_from("<i", u, 4)[0]
    text = text_fn(u[8:8 + lt])
    p = 8 + lt
    n = struct.unpack_from("<i", u, p)[0]
    q = p + 4
    for _ in range(n):
        q += 8 + struct.unpack_from("<i", u, q)[0]
    out = [b"BAM\x01", struct.pack("<i", len(text)), text, u[p:q]]
    i = 0
    while q + 4 <= len(u):
        bs = struct.unpack_from("<i", u, q)[0]
        r = u[q:q + 4 + bs]
        q += 4 + bs
        lrn, nc, ls = r[12], struct.unpack_from("<H", r, 16)[0], max(0, struct.unpack_from("<i", r, 20)[0])
        vstart = 36 + lrn + 4 * nc + (ls + 1) // 2 + ls
        items = oracle._aux_items(r[vstart:])
        aux, done = b"", False
        for tag, ty, val in items:
            if tag == b"RG" and not done:
                done = True
                new = rg_fn(i, val[:-1] if ty == b"Z" else val)
                if new is None:
                    continue
                if isinstance(new, tuple):
                    aux += tag + new[0] + new[1]
                else:
                    aux += tag + b"Z" + new + b"\0"
            else:
                aux += tag + ty + val
        body = bytearray(r[4:vstart] + aux)
        if ref_fn is not None:
            for o in (0, 20):  # refID, mate refID (body offsets)
                v = struct.unpack_from("<i", body, o)[0]
                if v >= 0:
                    struct.pack_into("<i", body, o, ref_fn(i, v))
        out.append(struct.pack("<i", len(body)) + bytes(body))
        i += 1
    return np.frombuffer(bgzf_pack(b"".join(out)), np.uint8).copy()


def reheader_bam(data, text_fn=None, refs_fn=None):
    """A copy of a BAM with its header rewritten: text_fn(text) -> new text, refs_fn(refs) -> new
    binary dictionary [(name bytes incl. anything after whitespace, l_ref)] (crafted-header tests
    of SAMHeaderReader / [htsjdk] BAMFileReader.readHeader); the records are kept as they are.
    A name given as (raw bytes, l_name) writes that l_name (e.g. 1: an empty name)."""
    import struct
    u = bam_stream(data)
    lt = struct.unpack_from("<i", u, 4)[0]
    text = u[8:8 + lt]
    p = 8 + lt
    n = struct.unpack_from("<i", u, p)[0]
    p += 4
    refs = []
    for _ in range(n):
        ln = struct.unpack_from("<i", u, p)[0]
        refs.append((u[p + 4:p + 3 + ln], struct.unpack_from("<i", u, p + 4 + ln)[0]))
        p += 8 + ln
    text = text_fn(text) if text_fn else text
    refs = refs_fn(refs) if refs_fn else refs
    out = [b"BAM\x01", struct.pack("<i", len(text)), text, struct.pack("<i", len(refs))]
    for nm, ln in refs:
        if isinstance(nm, tuple):
            raw, l_name = nm
            out += [struct.pack("<i", l_name), raw]
        else:
            out += [struct.pack("<i", len(nm) + 1), nm, b"\0"]
        out.append(struct.pack("<i", ln))
    out.append(u[p:])
    return np.frombuffer(bgzf_pack(b"".join(out)), np.uint8).copy()


def _sq_edit(k, fn):
    """text_fn editing the k-th @SQ line with fn(line) -> line"""
    def ed(text):
        lines = text.split(b"\n")
        idx = [i for i, ln in enumerate(lines) if ln.startswith(b"@SQ")]
        lines[idx[k]] = fn(lines[idx[k]])
        return b"\n".join(lines)
    return ed


# crafted headers: (label, text_fn, refs_fn, accepted by the reader?)
CRAFTED_HEADERS = [
    ("as_is", None, None, True),
    ("name_mismatch", None, lambda r: [(b"chrX" if i == 3 else nm, ln) for i, (nm, ln) in enumerate(r)], False),
    ("length_mismatch", None, lambda r: [(nm, ln + 1 if i == 7 else ln) for i, (nm, ln) in enumerate(r)], False),
    ("empty_name", None, lambda r: [((b"\0", 1) if i == 2 else nm, ln) for i, (nm, ln) in enumerate(r)], False),
    ("count_mismatch", None, lambda r: r[:-1], False),
    ("binary_name_cut_at_whitespace", None,
     lambda r: [(nm + b" extra words" if i == 4 else nm, ln) for i, (nm, ln) in enumerate(r)], True),
    ("no_sq_in_text", lambda t: b"\n".join(ln for ln in t.split(b"\n") if not ln.startswith(b"@SQ")), None, True),
    ("no_sq_in_text_any_binary", lambda t: b"\n".join(ln for ln in t.split(b"\n") if not ln.startswith(b"@SQ")),
     lambda r: [(b"zz" + nm, 7) for nm, _ in r], True),
    ("sq_without_ln", None, None, False),  # text_fn set below
    ("sq_ln_not_an_int", None, None, False),
    ("crlf_lines", lambda t: t.replace(b"\n", b"\r\n"), None, True),
]
CRAFTED_HEADERS[8] = ("sq_without_ln", _sq_edit(1, lambda ln: b"\t".join(
    f for f in ln.split(b"\t") if not f.startswith(b"LN:"))), None, False)
CRAFTED_HEADERS[9] = ("sq_ln_not_an_int", _sq_edit(0, lambda ln: ln.replace(b"LN:", b"LN:x")), None, False)
