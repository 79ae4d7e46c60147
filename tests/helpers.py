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
