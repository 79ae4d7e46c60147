"""ctypes wrapper of the CPU oracle (liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this,
and only as the checker / the timed CPU baseline.  The product path (libhbam.so)
never loads it.  Parity status is documented in hbam_oracle.h and DESIGN.md §3.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

OR_OK, OR_EIO, OR_ETRUNC, OR_EFORMAT, OR_ERUNTIMEIO, OR_EEOF, OR_EREFID, OR_EDATA, OR_ENOMEM = (
    0, -1, -2, -3, -4, -5, -6, -7, -8)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        u8p = C.POINTER(C.c_uint8)
        L.or_murmurhash3.restype = C.c_int64
        L.or_murmurhash3.argtypes = [u8p, C.c_int32, C.c_int32]
        L.or_get_key.restype = C.c_int64
        L.or_get_key.argtypes = [C.c_int32, C.c_int32, C.c_uint16, u8p, C.c_int32]
        L.or_scan_blocks.restype = C.c_int64
        L.or_scan_blocks.argtypes = [u8p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
        L.or_inflate_block.restype = C.c_int
        L.or_inflate_block.argtypes = [u8p, C.c_uint32, C.c_void_p, C.c_uint32,
                                       C.POINTER(C.c_uint32), C.c_int]
        L.or_read_header.restype = C.c_int
        L.or_read_header.argtypes = [u8p, C.c_uint64, C.POINTER(OrHeader)]
        L.or_guess_bam_record_start.restype = C.c_int64
        L.or_guess_bam_record_start.argtypes = [u8p, C.c_uint64, C.c_int64, C.c_int64, C.c_int32,
                                                C.POINTER(C.c_int)]
        L.or_guess_bgzf_block_start.restype = C.c_int64
        L.or_guess_bgzf_block_start.argtypes = [u8p, C.c_uint64, C.c_int64, C.c_int64,
                                                C.POINTER(C.c_int)]
        L.or_file_splits.restype = C.c_int64
        L.or_file_splits.argtypes = [C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64]
        L.or_probabilistic_splits.restype = C.c_int64
        L.or_probabilistic_splits.argtypes = [u8p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64,
                                              C.c_void_p, C.c_void_p]
        L.or_splitting_index.restype = C.c_int64
        L.or_splitting_index.argtypes = [u8p, C.c_uint64, C.c_int32, C.c_void_p, C.c_uint64]
        L.or_bgzf_block_index.restype = C.c_int64
        L.or_bgzf_block_index.argtypes = [u8p, C.c_uint64, C.c_int32, C.c_void_p, C.c_uint64]
        L.or_read_split_cols_nref.restype = C.c_int
        L.or_read_split_cols_nref.argtypes = [u8p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, C.c_int,
                                              C.c_int32, C.POINTER(OrCols)]
        L.or_read_split_cols.restype = C.c_int
        L.or_read_split_cols.argtypes = [u8p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, C.c_int,
                                         C.POINTER(OrCols)]
        L.or_read_split_pools.restype = C.c_int
        L.or_read_split_pools.argtypes = [u8p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int32,
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.or_probabilistic_splits_nref.restype = C.c_int64
        L.or_probabilistic_splits_nref.argtypes = [u8p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64,
                                                   C.c_int32, C.c_void_p, C.c_void_p]
        L.or_check_split.restype = C.c_int
        L.or_check_split.argtypes = [u8p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int32, C.c_void_p,
                                     C.c_uint64, C.c_void_p]
        L.or_cols_free.restype = None
        L.or_cols_free.argtypes = [C.POINTER(OrCols)]
        vp = C.c_void_p
        L.or_summarize_ranges.restype = C.c_int64
        L.or_summarize_ranges.argtypes = [vp, vp, C.c_uint64, C.c_int32, vp, vp, vp, vp, vp,
                                          C.c_uint64, C.POINTER(C.c_int32)]
        L.or_name_order.restype = None
        L.or_name_order.argtypes = [vp, vp, C.c_uint64, vp]
        L.or_fixmate.restype = C.c_int64
        L.or_fixmate.argtypes = [vp, vp, C.c_uint64, vp, vp, vp, C.c_uint64, C.c_uint64,
                                 C.POINTER(C.c_int32)]
        L.or_bcf_read_header.restype = C.c_int
        L.or_bcf_read_header.argtypes = [u8p, C.c_uint64, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                         C.POINTER(C.c_int32), C.POINTER(C.c_uint64)]
        L.or_guess_bcf_record_start.restype = C.c_int64
        L.or_guess_bcf_record_start.argtypes = [u8p, C.c_uint64, C.c_int64, C.c_int64, C.c_int,
                                                C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int)]
        L.or_read_bcf_split.restype = C.c_int64
        L.or_read_bcf_split.argtypes = [u8p, C.c_uint64, C.c_int, C.c_uint64, C.c_uint64, C.c_int32,
                                        C.c_int32, C.c_int32, C.c_uint64, vp, vp, vp, vp, C.c_uint64,
                                        C.POINTER(C.c_int)]
        _LIB = L
    return _LIB


class OrHeader(C.Structure):
    _fields_ = [("l_text", C.c_int32), ("n_ref", C.c_int32), ("header_ulen", C.c_uint64),
                ("first_voffset", C.c_uint64)]


class OrCols(C.Structure):
    _fields_ = [("n", C.c_uint64), ("status", C.c_int32), ("err_record", C.c_uint64),
                ("voffset", C.POINTER(C.c_uint64)), ("key", C.POINTER(C.c_int64)),
                ("block_size", C.POINTER(C.c_int32)), ("ref_id", C.POINTER(C.c_int32)),
                ("pos", C.POINTER(C.c_int32)), ("l_read_name", C.POINTER(C.c_uint8)),
                ("mapq", C.POINTER(C.c_uint8)), ("bin", C.POINTER(C.c_uint16)),
                ("n_cigar", C.POINTER(C.c_uint16)), ("flag", C.POINTER(C.c_uint16)),
                ("l_seq", C.POINTER(C.c_int32)), ("next_ref_id", C.POINTER(C.c_int32)),
                ("next_pos", C.POINTER(C.c_int32)), ("tlen", C.POINTER(C.c_int32)),
                ("var_off", C.POINTER(C.c_uint64)), ("var", C.POINTER(C.c_uint8)),
                ("cap", C.c_uint64), ("var_cap", C.c_uint64)]


FIXED_FIELDS = [("voffset", np.uint64), ("key", np.int64), ("block_size", np.int32),
                ("ref_id", np.int32), ("pos", np.int32), ("l_read_name", np.uint8),
                ("mapq", np.uint8), ("bin", np.uint16), ("n_cigar", np.uint16),
                ("flag", np.uint16), ("l_seq", np.int32), ("next_ref_id", np.int32),
                ("next_pos", np.int32), ("tlen", np.int32)]


def _buf(data):
    """uint8 pointer to a bytes-like / numpy buffer (kept alive by the caller)."""
    a = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return a, a.ctypes.data_as(C.POINTER(C.c_uint8))


def murmurhash3(b, seed=0):
    a, p = _buf(bytes(b) if len(b) else b"\0")
    return lib().or_murmurhash3(p, len(b), seed)


def get_key(ref_id, pos0, flag, var):
    a, p = _buf(bytes(var) if len(var) else b"\0")
    return lib().or_get_key(ref_id, pos0, flag, p, len(var))


def scan_blocks(data):
    a, p = _buf(data)
    cap = len(a) // 26 + 2
    coff = np.zeros(cap, np.uint64)
    clen = np.zeros(cap, np.uint32)
    isz = np.zeros(cap, np.uint32)
    crc = np.zeros(cap, np.uint32)
    bad = C.c_uint64(0)
    n = lib().or_scan_blocks(p, len(a), coff.ctypes.data, clen.ctypes.data, isz.ctypes.data,
                             crc.ctypes.data, cap, C.byref(bad))
    if n < 0:
        return n, int(bad.value)
    return dict(coff=coff[:n], clen=clen[:n], isize=isz[:n], crc=crc[:n])


def inflate_block(blk, check_crc=True):
    a, p = _buf(blk)
    out = np.zeros(1 << 16, np.uint8)
    ol = C.c_uint32(0)
    rc = lib().or_inflate_block(p, len(a), out.ctypes.data, len(out), C.byref(ol), int(check_crc))
    return rc, bytes(out[:ol.value]) if rc == 0 else b""


def read_header(data):
    a, p = _buf(data)
    h = OrHeader()
    rc = lib().or_read_header(p, len(a), C.byref(h))
    if rc:
        return rc
    return dict(l_text=h.l_text, n_ref=h.n_ref, header_ulen=h.header_ulen,
                first_voffset=h.first_voffset)


def read_split(data, v_start, v_end, check_crc=False, keep_var=True, n_ref=None):
    """BAMRecordReader over one FileVirtualSplit -> dict of numpy columns.  n_ref given: `data` is a
    window of the file (a byte-range shard, voffsets relative to it) whose header was read elsewhere."""
    a, p = _buf(data)
    c = OrCols()
    if n_ref is None:
        lib().or_read_split_cols(p, len(a), v_start, v_end, int(check_crc), int(keep_var), C.byref(c))
    else:
        lib().or_read_split_cols_nref(p, len(a), v_start, v_end, int(check_crc), int(keep_var), int(n_ref),
                                      C.byref(c))
    n = int(c.n)
    out = dict(n=n, status=int(c.status), err_record=int(c.err_record))
    for name, dt in FIXED_FIELDS:
        ptr = getattr(c, name)
        out[name] = (np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt).copy() if n
                     else np.zeros(0, dt))
    out["var_off"] = np.ctypeslib.as_array(c.var_off, shape=(n + 1,)).copy()
    vl = int(out["var_off"][-1])
    out["var"] = np.ctypeslib.as_array(c.var, shape=(vl,)).copy() if vl else np.zeros(0, np.uint8)
    lib().or_cols_free(C.byref(c))
    return out


def guess_bam_record_start(data, beg, end, n_ref):
    a, p = _buf(data)
    err = C.c_int(0)
    r = lib().or_guess_bam_record_start(p, len(a), beg, end, n_ref, C.byref(err))
    return r, err.value


def guess_bgzf_block_start(data, beg, end):
    a, p = _buf(data)
    err = C.c_int(0)
    r = lib().or_guess_bgzf_block_start(p, len(a), beg, end, C.byref(err))
    return r, err.value


def file_splits(file_len, split_size):
    cap = file_len // max(split_size, 1) + 4
    b = np.zeros(cap, np.uint64)
    e = np.zeros(cap, np.uint64)
    n = lib().or_file_splits(file_len, split_size, b.ctypes.data, e.ctypes.data, cap)
    return b[:n], e[:n]


def probabilistic_splits(data, beg, end):
    a, p = _buf(data)
    beg = np.ascontiguousarray(beg, np.uint64)
    end = np.ascontiguousarray(end, np.uint64)
    vs = np.zeros(len(beg), np.uint64)
    ve = np.zeros(len(beg), np.uint64)
    n = lib().or_probabilistic_splits(p, len(a), beg.ctypes.data, end.ctypes.data, len(beg),
                                      vs.ctypes.data, ve.ctypes.data)
    if n < 0:
        return n
    return vs[:n], ve[:n]


def probabilistic_splits_nref(data, beg, end, n_ref):
    """addProbabilisticSplits over a window of the file (no header in `data`)"""
    a, p = _buf(data)
    beg = np.ascontiguousarray(beg, np.uint64)
    end = np.ascontiguousarray(end, np.uint64)
    vs = np.zeros(len(beg), np.uint64)
    ve = np.zeros(len(beg), np.uint64)
    n = lib().or_probabilistic_splits_nref(p, len(a), beg.ctypes.data, end.ctypes.data, len(beg), n_ref,
                                           vs.ctypes.data, ve.ctypes.data)
    if n < 0:
        return n
    return vs[:n], ve[:n]


class OrDevCols(C.Structure):
    _fields_ = [("n", C.c_uint64), ("voff_base", C.c_uint64)] + [
        (k, C.c_void_p) for k in ("voffset", "key", "rec_off", "ubuf")] + [("ubuf_len", C.c_uint64)] + [
        (k, C.c_void_p) for k in ("block_size", "ref_id", "pos", "l_read_name", "mapq", "bin", "n_cigar",
                                  "flag", "l_seq", "next_ref_id", "next_pos", "tlen", "layout_ok",
                                  "name_off", "cigar_off", "seq_off", "aux_off", "names", "cigars",
                                  "seq", "qual", "aux")]


class OrCheck(C.Structure):
    _fields_ = [("n_checked", C.c_uint64), ("mismatches", C.c_uint64), ("first_bad", C.c_int64),
                ("bad_field", C.c_int32), ("status", C.c_int32)]


CHECK_FIELDS = {1: "count", 2: "voffset", 3: "key", 4: "fixed", 5: "record bytes", 6: "layout_ok",
                7: "names", 8: "cigars", 9: "seq", 10: "qual", 11: "aux"}


def check_whole(data, own_len, n_ref, dev, voff_base, n_splits, threads):
    """Every record of one device decode checked against the oracle (test infrastructure:
    bench.py's at-size parity).  `data` is the compressed window the device decoded, its
    FileSplit [0, own_len): the device's FileVirtualSplit is [guess(0), own_len << 16 | 0xffff).
    `dev` is an OrDevCols over the decode's host copy, record i at index i, voffsets = window
    voffsets + voff_base.  The oracle's own guess of 0 must be the device's first record; the
    sequential read is then cut at the device's voffsets of every (n / n_splits)-th record, and
    the pieces are read by the oracle's BAMRecordReader one per thread and compared record by
    record with the device records (C, or_check_split).  A piece that starts at a device voffset
    that is not a true record start, or a device record missing or extra, shows up as a count
    or voffset mismatch of the piece before it, so the pieces tile the read exactly."""
    import threading
    a, p = _buf(data)
    n = int(dev.n)
    out = {"shard_records": n, "records_checked": 0}
    g, err = guess_bam_record_start(a, 0, own_len, n_ref)
    dvo = np.ctypeslib.as_array(C.cast(dev.voffset, C.POINTER(C.c_uint64)), shape=(n,)) \
        if n else np.zeros(0, np.uint64)
    if err or g == own_len or not n or int(dvo[0]) != g + voff_base:
        out["error"] = "first record: oracle guess %d (err %d), device %s" % (
            g, err, int(dvo[0]) - voff_base if n else None)
        return out
    S = max(1, min(n_splits, n))
    idx = np.array([n * k // S for k in range(S + 1)], np.int64)
    vs = [int(dvo[idx[k]]) - voff_base for k in range(S)]
    ve = vs[1:] + [(own_len << 16) | 0xffff]
    outs = [OrCheck() for _ in range(S)]
    L = lib()

    def work(k):
        L.or_check_split(p, len(a), vs[k], ve[k], n_ref, C.addressof(dev), int(idx[k]), C.addressof(outs[k]))

    ths = [threading.Thread(target=work, args=(k,)) for k in range(S)]
    for k in range(0, S, max(1, threads)):
        for th in ths[k:k + threads]:
            th.start()
        for th in ths[k:k + threads]:
            th.join()
    short = [k for k in range(S) if int(outs[k].n_checked) != int(idx[k + 1] - idx[k])]
    bad = [k for k in range(S) if outs[k].mismatches]
    out.update({
        "records_checked": int(sum(min(int(o.n_checked), int(idx[k + 1] - idx[k])) for k, o in enumerate(outs))),
        "pieces": S, "pieces_with_wrong_count": len(short),
        "mismatches": int(sum(o.mismatches for o in outs)) + len(short),
        "oracle_status": sorted(set(int(o.status) for o in outs)),
        "first_bad": ({"record": int(outs[bad[0]].first_bad),
                       "field": CHECK_FIELDS.get(int(outs[bad[0]].bad_field), "?")} if bad else
                      {"record": int(idx[short[0]]), "field": "count"} if short else None)})
    return out


def splitting_index(data, granularity=4096):
    a, p = _buf(data)
    cap = 1 << 20
    out = np.zeros(cap, np.uint64)
    n = lib().or_splitting_index(p, len(a), granularity, out.ctypes.data, cap)
    if n < 0:
        return n
    return out[:n]


def bgzf_block_index(data, granularity=1):
    """BGZFBlockIndexer.index (util/BGZFBlockIndexer.java:97-181): u64 entries (48-bit
    values) or a negative code."""
    a, p = _buf(data)
    cap = len(a) // 28 + 2
    out = np.zeros(cap, np.uint64)
    n = lib().or_bgzf_block_index(p, len(a), granularity, out.ctypes.data, cap)
    if n < 0:
        return n
    return out[:n]


# ---- Sort plugin path (Sort.java:84-188) --------------------------------------------------
_REC_DT = np.dtype([("block_size", "<i4"), ("ref_id", "<i4"), ("pos", "<i4"),
                    ("l_read_name", "u1"), ("mapq", "u1"), ("bin", "<u2"), ("n_cigar", "<u2"),
                    ("flag", "<u2"), ("l_seq", "<i4"), ("next_ref_id", "<i4"), ("next_pos", "<i4"),
                    ("tlen", "<i4")])


def record_fixed_bytes(cols, idx):
    """the 36 fixed bytes (block_size .. tlen) of records idx of a read_split result: (k, 36) u8"""
    idx = np.asarray(idx, np.int64)
    fixed = np.zeros(len(idx), _REC_DT)
    for f in _REC_DT.names:
        fixed[f] = cols[f][idx]
    return fixed.view(np.uint8).reshape(len(idx), 36)


def record_payloads(cols):
    """SAMRecordWritable.write (SAMRecordWritable.java:62-63: BAMRecordCodec.encode of an
    untouched lazily-decoded record = its block_size + original bytes) for every record of a
    read_split result -> (payload uint8, offsets int64[n+1])."""
    n = cols["n"]
    fixed = np.zeros(n, _REC_DT)
    for f in _REC_DT.names:
        fixed[f] = cols[f]
    fb = fixed.view(np.uint8).reshape(n, 36)
    vo = cols["var_off"].astype(np.int64)
    lens = 36 + (vo[1:] - vo[:-1])
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(lens)
    out = np.zeros(int(off[-1]), np.uint8)
    for i in range(n):
        o = int(off[i])
        out[o:o + 36] = fb[i]
        out[o + 36:int(off[i + 1])] = cols["var"][int(vo[i]):int(vo[i + 1])]
    return out, off


_SEQ_ALPHA = np.frombuffer(b"=ACMGRSVTWYHKDBN", dtype=np.uint8)


def _gather(src, starts, lens):
    """concatenation of src[starts[i]:starts[i]+lens[i]] over i (vectorised)"""
    lens = np.asarray(lens, np.int64)
    tot = int(lens.sum())
    if tot == 0:
        return np.zeros(0, src.dtype), np.zeros(0, np.int64)
    excl = np.cumsum(lens) - lens
    k = np.arange(tot, dtype=np.int64) - np.repeat(excl, lens)  # index inside the segment
    return src[np.repeat(np.asarray(starts, np.int64), lens) + k], k


def pools(cols):
    """The lazy getters' decoded fields of every record of a read_split result, concatenated in
    record order (BAMRecord.getReadName / getCigar / getReadBases / getBaseQualities /
    attributes): read names incl. NUL, CIGAR u32s, SEQ as
    "=ACMGRSVTWYHKDBN" characters (high nibble first), QUAL, AUX bytes; plus layout_ok (the
    variable block holds name + CIGAR + SEQ + QUAL).  Vectorised numpy (tests/helpers.py
    has a per-record loop form of the same)."""
    var = cols["var"]
    vo = cols["var_off"].astype(np.int64)
    L = cols["l_read_name"].astype(np.int64)
    nc = cols["n_cigar"].astype(np.int64)
    ls = cols["l_seq"].astype(np.int64)
    vlen = vo[1:] - vo[:-1]
    fixed = L + 4 * nc + (ls + 1) // 2 + ls
    ok = (ls >= 0) & (fixed <= vlen)
    L, nc, ls = np.where(ok, L, 0), np.where(ok, nc, 0), np.where(ok, ls, 0)
    na = np.where(ok, vlen - fixed, 0)
    s_name = vo[:-1]
    s_cig = s_name + L
    s_seq = s_cig + 4 * nc
    s_qual = s_seq + (ls + 1) // 2
    s_aux = s_qual + ls
    names, _ = _gather(var, s_name, L)
    cig, _ = _gather(var, s_cig, 4 * nc)
    packed, k = _gather(var, s_seq, ls)  # one entry per character: k = character index
    byte = var[np.repeat(s_seq, ls) + k // 2] if len(k) else np.zeros(0, np.uint8)
    nib = np.where(k % 2 == 0, byte >> 4, byte & 15)
    qual, _ = _gather(var, s_qual, ls)
    aux, _ = _gather(var, s_aux, na)
    return dict(layout_ok=ok.astype(np.uint8), names=names.astype(np.uint8),
                cigars=np.ascontiguousarray(cig.astype(np.uint8)).view(np.uint32),
                seq=_SEQ_ALPHA[nib] if len(nib) else np.zeros(0, np.uint8),
                qual=qual.astype(np.uint8), aux=aux.astype(np.uint8))


def sort_order(keys):
    """Sort's total order over LongWritable keys (signed i64 comparator, Sort.java:149-157 +
    TotalOrderPartitioner; identity reduce).  The reference leaves ties unspecified; the
    documented order is input order (key, file, voffset): a stable sort."""
    return np.argsort(np.asarray(keys, np.int64), kind="stable")


class CpuSortOps:
    """The Sort exchange's local ops on CPU tensors, restated with numpy (tests' gloo runs)."""

    @staticmethod
    def run_from_arrays(keys, voffset, block_size, payload, offsets):
        import torch
        o = sort_order(keys)
        new_off, pay = _regather(payload, offsets, o)
        from hadoop_bam.sort import SortedRun
        return SortedRun(torch.from_numpy(np.asarray(keys, np.int64)[o].copy()),
                         torch.from_numpy(np.asarray(voffset).astype(np.int64)[o].copy()),
                         torch.from_numpy(np.asarray(block_size, np.int32)[o].copy()),
                         torch.from_numpy(pay), torch.from_numpy(new_off))

    @staticmethod
    def sort_received(keys, voffset, block_size, payload):
        bs = block_size.numpy().astype(np.int64)
        off = np.zeros(len(bs) + 1, np.int64)
        off[1:] = np.cumsum(4 + bs)
        return CpuSortOps.run_from_arrays(keys.numpy(), voffset.numpy(), block_size.numpy(),
                                          payload.numpy(), off)


def _regather(payload, offsets, order):
    offsets = np.asarray(offsets, np.int64)
    lens = (offsets[1:] - offsets[:-1])[order]
    new_off = np.zeros(len(order) + 1, np.int64)
    new_off[1:] = np.cumsum(lens)
    out = np.zeros(int(new_off[-1]), np.uint8)
    for j, i in enumerate(order):
        out[new_off[j]:new_off[j + 1]] = payload[offsets[i]:offsets[i + 1]]
    return new_off, out


# ---- multi-input Sort (Sort.java:111-113, 279-295; cli/Utils.java:252-325) -----------------
def bam_dictionary(data):
    """The sequence dictionary [(name, length)] of a BAM (zlib over the first members)."""
    import struct
    import zlib
    d = bytes(np.asarray(data, np.uint8)[:64 << 20])
    u, p = b"", 0
    while p + 18 <= len(d):
        bs = struct.unpack_from("<H", d, p + 16)[0] + 1
        u += zlib.decompressobj(-15).decompress(d[p + 18:p + bs - 8])
        p += bs
        if len(u) >= 12:
            lt = struct.unpack_from("<i", u, 4)[0]
            q = 8 + lt
            if len(u) >= q + 4:
                n = struct.unpack_from("<i", u, q)[0]
                q += 4
                out, ok = [], True
                for _ in range(n):
                    if len(u) < q + 4:
                        ok = False
                        break
                    ln = struct.unpack_from("<i", u, q)[0]
                    if len(u) < q + 8 + ln:
                        ok = False
                        break
                    out.append((u[q + 4:q + 3 + ln], struct.unpack_from("<i", u, q + 4 + ln)[0]))
                    q += 8 + ln
                if ok:
                    return out
    raise ValueError("truncated header")


def merged_dictionary(dicts):
    """SamFileHeaderMerger (htsjdk 1.131, mergeDictionaries = true; restated, parity unpinned):
    -> (merged [(name, len)], merged?) — inputs folded left to right by mergeSequences."""
    def same(a, b):
        return len(a) == len(b) and all(x[0] == y[0] and (x[1] == y[1] or not x[1] or not y[1])
                                        for x, y in zip(a, b))
    if all(same(dicts[0], d) for d in dicts[1:]):
        return list(dicts[0]), False
    acc = []
    for frm in dicts:
        res = list(acc)
        held = []
        last = -1
        for rec in frm:
            at = next((k for k, r in enumerate(res) if r[0] == rec[0]), -1)
            if at < 0:
                held.append(rec)
                continue
            if at < last:
                raise ValueError("sequence dictionaries in different orders")
            res = res[:at] + held + res[at:]
            last = at + len(held)
            held = []
        acc = res + held
    return acc, True


def correct_payloads(pay, off, keys, ref_map):
    """Utils.correctSAMRecordForMerging + SortRecordReader's re-key on SAMRecordWritable
    payloads (copy): refID -> ref_map, next refID too for paired reads, the coordinate key
    recomputed where refID changed.  -> (payload, keys, first record raising or -1)."""
    import struct
    pay = np.array(pay, np.uint8, copy=True)
    keys = np.array(keys, np.int64, copy=True)
    n_in = len(ref_map)
    for i in range(len(off) - 1):
        o = int(off[i])
        ref, pos = struct.unpack_from("<ii", pay, o + 4)
        flag = struct.unpack_from("<H", pay, o + 18)[0]
        mref = struct.unpack_from("<i", pay, o + 24)[0]

        def tr(x):
            return -1 if x == -1 else (int(ref_map[x]) if 0 <= x < n_in else n_in)
        nr = tr(ref)
        nm = tr(mref) if flag & 1 else mref
        if nr >= n_in or nm >= n_in:
            return pay, keys, i
        if nr != ref:
            struct.pack_into("<i", pay, o + 4, nr)
            if not (flag & 4) and nr >= 0 and np.int32(pos + 1) >= 0:
                keys[i] = (nr << 32) | pos  # getKey0: the int pos sign-extended before the OR
        if nm != mref:
            struct.pack_into("<i", pay, o + 24, nm)
    return pay, keys, -1


def bam_header_text(data):
    """The SAM text of a BAM header (zlib over the first members)."""
    import struct
    import zlib
    d = bytes(np.asarray(data, np.uint8)[:64 << 20])
    u, p = b"", 0
    while p + 18 <= len(d):
        bs = struct.unpack_from("<H", d, p + 16)[0] + 1
        u += zlib.decompressobj(-15).decompress(d[p + 18:p + bs - 8])
        p += bs
        if len(u) >= 8 and len(u) >= 8 + struct.unpack_from("<i", u, 4)[0]:
            return u[8:8 + struct.unpack_from("<i", u, 4)[0]]
    raise ValueError("truncated header")


def _group_lines(text, tag):
    recs = []
    for ln in text.split(b"\n"):
        if not ln.startswith(tag + b"\t"):
            continue
        fields = {}
        order = []
        for f in ln.split(b"\t")[1:]:
            if len(f) < 3:
                continue
            if f[:2] not in fields:
                order.append(f[:2])
            fields[f[:2]] = f[3:]
        recs.append((fields.get(b"ID", b""), fields, order))
    return recs


def _merge_records(pairs, taken, translation):
    """SamFileHeaderMerger.mergeHeaderRecords (htsjdk 1.131; restated: parity unpinned)."""
    groups = []  # [(id, [(attrs-without-ID, [input])])] in first-seen order
    for inp, rid, fields in pairs:
        attrs = {k: v for k, v in fields.items() if k != b"ID"}
        g = next((x for x in groups if x[0] == rid), None)
        if g is None:
            g = (rid, [])
            groups.append(g)
        v = next((x for x in g[1] if x[0] == attrs), None)
        if v is None:
            v = (attrs, [])
            g[1].append(v)
        v[1].append(inp)
    collision = False
    merged = []
    for rid, variants in groups:
        for attrs, inputs in variants:
            if rid in taken:
                collision = True
                i = 1
                while (rid + b".%d" % i) in taken:
                    i += 1
                new = rid + b".%d" % i
            else:
                new = rid
            taken.add(new)
            for inp in inputs:
                translation.setdefault(inp, {})[rid] = new
            merged.append((new, attrs))
    return collision, merged


def header_groups(texts):
    """mergeReadGroups / mergeProgramGroups over the inputs' header texts -> dict(rg_collisions,
    pg_collisions, rg (per-input id translation), pg (per-input; absent = no @PG record))."""
    for t in texts:
        for tag in (b"@RG", b"@PG"):
            ids = [r[0] for r in _group_lines(t, tag)]
            if len(set(ids)) != len(ids):
                raise ValueError("duplicate %s id in one input" % tag.decode())
    rg_tr = {}
    rg_col, _ = _merge_records([(i, rid, f) for i, t in enumerate(texts) for rid, f, _ in _group_lines(t, b"@RG")],
                               set(), rg_tr)
    pending = [(i, rid, dict(f)) for i, t in enumerate(texts) for rid, f, _ in _group_lines(t, b"@PG")]
    current = [x for x in pending if b"PP" not in x[2]]
    pending = [x for x in pending if b"PP" in x[2]]
    taken, pg_tr, pg_col = set(), {}, False
    while current:
        c, _ = _merge_records(current, taken, pg_tr)
        pg_col = pg_col or c
        current = [(i, pg_tr.get(i, {}).get(rid, rid), f) for i, rid, f in current]
        moved = []
        for i, rid, f in pending:
            f = dict(f)
            t = pg_tr.get(i, {})
            if f[b"PP"] in t:
                f[b"PP"] = t[f[b"PP"]]
            moved.append((i, rid, f))
        pending = moved
        current, pending = ([x for x in pending if any(x[0] == y[0] and x[2][b"PP"] == y[1] for y in current)],
                            [x for x in pending if not any(x[0] == y[0] and x[2][b"PP"] == y[1] for y in current)])
    if pending:
        raise ValueError("program groups whose PP points nowhere")
    return {"rg_collisions": rg_col, "pg_collisions": pg_col, "rg": rg_tr, "pg": pg_tr}


class GroupRewriteError(Exception):
    def __init__(self, kind, record):
        super().__init__("%s at record %d" % (kind, record))
        self.kind, self.record = kind, record


def _aux_items(aux):
    """[(tag, type, value bytes)] of a BAM aux block; raises ValueError if it does not parse."""
    import struct
    out, p = [], 0
    sizes = {b"A": 1, b"c": 1, b"C": 1, b"s": 2, b"S": 2, b"i": 4, b"I": 4, b"f": 4}
    while p < len(aux):
        if len(aux) - p < 3:
            raise ValueError("aux")
        tag, ty = aux[p:p + 2], aux[p + 2:p + 3]
        q = p + 3
        if ty in sizes:
            n = sizes[ty]
        elif ty in (b"Z", b"H"):
            z = aux.find(b"\0", q)
            if z < 0:
                raise ValueError("aux")
            n = z - q + 1
        elif ty == b"B":
            if len(aux) - q < 5:
                raise ValueError("aux")
            st = aux[q:q + 1]
            es = {b"c": 1, b"C": 1, b"s": 2, b"S": 2, b"i": 4, b"I": 4, b"f": 4}.get(st)
            if es is None:
                raise ValueError("aux")
            n = 5 + es * struct.unpack_from("<I", aux, q + 1)[0]
        else:
            raise ValueError("aux")
        if q + n > len(aux):
            raise ValueError("aux")
        out.append((tag, ty, aux[q:q + n]))
        p = q + n
    return out


def _int_type(v):
    """BinaryTagCodec.getIntegerType"""
    if v > 2147483647:
        return b"I"
    if v > 65535:
        return b"i"
    if v > 255:
        return b"S"
    if v > 127:
        return b"C"
    if v >= -128:
        return b"c"
    if v >= -32768:
        return b"s"
    return b"i"


def rewrite_group_tags(pay, off, groups, inp):
    """Utils.correctSAMRecordForMerging's PG / RG rewrite (cli/Utils.java:314-324) of input `inp`'s
    SAMRecordWritable payloads, and BAMRecordCodec.encode of every record on which setAttribute ran
    (htsjdk 1.131 restated, parity unpinned: integers re-typed, pad nibble 0, absent qualities
    0xFF, bin 0 when unplaced; a replaced tag keeps its place).  -> (payload, offsets); raises
    GroupRewriteError(kind, record) where the reference's map task fails."""
    import struct
    pg_map = groups["pg"].get(inp)  # the RG lookup uses the PROGRAM-group table too (:322)
    todo = [t for t, c in ((b"PG", groups["pg_collisions"]), (b"RG", groups["rg_collisions"])) if c]
    out = []
    for i in range(len(off) - 1):
        r = bytes(pay[int(off[i]):int(off[i + 1])])
        if not todo:
            out.append(r)
            continue
        lrn, nc, ls = r[12], struct.unpack_from("<H", r, 16)[0], max(0, struct.unpack_from("<i", r, 20)[0])
        head = 36 + lrn + 4 * nc
        vstart = head + (ls + 1) // 2 + ls
        try:
            items = _aux_items(r[vstart:])
        except ValueError:
            raise GroupRewriteError("SAMFormatException", i)
        edits = {}
        for t in todo:
            first = next((k for k, it in enumerate(items) if it[0] == t), None)
            if first is None:
                continue
            if items[first][1] != b"Z":
                raise GroupRewriteError("ClassCastException", i)
            if pg_map is None:
                raise GroupRewriteError("NullPointerException", i)
            edits[first] = pg_map.get(items[first][2][:-1])
        if not edits:
            out.append(r)
            continue
        aux = b""
        for k, (tag, ty, val) in enumerate(items):
            if k in edits:
                if edits[k] is not None:
                    aux += tag + b"Z" + edits[k] + b"\0"
            elif ty in (b"c", b"C", b"s", b"S", b"i", b"I"):
                v = struct.unpack("<" + {b"c": "b", b"C": "B", b"s": "h", b"S": "H", b"i": "i", b"I": "I"}[ty], val)[0]
                nt = _int_type(v)
                aux += tag + nt + struct.pack("<" + {b"c": "b", b"C": "B", b"s": "h", b"S": "H", b"i": "i", b"I": "I"}[nt], v)
            else:
                aux += tag + ty + val
        seq = bytearray(r[head:head + (ls + 1) // 2])
        if ls & 1:
            seq[-1] &= 0xF0
        qual = r[head + (ls + 1) // 2:vstart]
        if ls and qual[0] == 0xFF:
            qual = b"\xff" * ls
        fixed = bytearray(r[:head])
        if struct.unpack_from("<i", r, 4)[0] < 0:
            struct.pack_into("<H", fixed, 14, 0)
        body = bytes(fixed[4:]) + bytes(seq) + qual + aux
        out.append(struct.pack("<i", len(body)) + body)
    offs = np.zeros(len(out) + 1, np.int64)
    offs[1:] = np.cumsum([len(x) for x in out])
    return np.frombuffer(b"".join(out), np.uint8), offs


def sort_merged(datas):
    """The multi-input Sort's total order over whole-file reads of every input: (key, input
    index, voffset) -> (keys, payload, offsets, merged dictionary)."""
    dicts = [bam_dictionary(d) for d in datas]
    merged, did = merged_dictionary(dicts)
    names = [n for n, _ in merged]
    groups = header_groups([bam_header_text(d) for d in datas])
    K, P, O, F, V = [], [], [], [], []
    for fi, (d, dic) in enumerate(zip(datas, dicts)):
        h = read_header(d)
        cols = read_split(d, h["first_voffset"], (len(d) << 16) | 0xffff)
        pay, off = record_payloads(cols)
        keys = cols["key"].astype(np.int64)
        if did:
            pay, keys, bad = correct_payloads(pay, off, keys, [names.index(n) for n, _ in dic])
            if bad >= 0:
                # correctSAMRecordForMerging runs per record (cli/Utils.java:286-324, called from
                # SortRecordReader.nextKeyValue, Sort.java:279-295): the records before `bad` get
                # their group step first, and an exception there comes first
                rewrite_group_tags(pay, off[:bad + 1], groups, fi)
                raise ValueError("input %d record %d: index outside its dictionary" % (fi, bad))
        pay, off = rewrite_group_tags(pay, off, groups, fi)
        for i in range(cols["n"]):
            P.append(bytes(pay[int(off[i]):int(off[i + 1])]))
        K.append(keys)
        F.append(np.full(cols["n"], fi, np.int64))
        V.append(cols["voffset"].astype(np.int64))
    keys = np.concatenate(K)
    o = np.lexsort((np.concatenate(V), np.concatenate(F), keys))
    pays = [P[i] for i in o]
    offs = np.zeros(len(o) + 1, np.int64)
    offs[1:] = np.cumsum([len(x) for x in pays])
    return keys[o], np.frombuffer(b"".join(pays), np.uint8), offs, merged


# ---- read-name / CIGAR keyed consumers ---------------------------------
def _pay(payload, offsets):
    pay = np.ascontiguousarray(payload, np.uint8)
    if pay.size == 0:
        pay = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(offsets, np.uint64)
    return pay, off, len(off) - 1


def summarize_ranges(payload, offsets, split_status=0):
    """SummarizeRecordReader (Summarize.java:664-755) over packed record payloads -> dict(key,
    beg, end, rev, record, status)."""
    pay, off, n = _pay(payload, offsets)
    cap = 1
    for i in range(n):  # upper bound: one range per CIGAR op + 1
        cap += int(pay[int(off[i]) + 16]) | int(pay[int(off[i]) + 17]) << 8
    cap += n
    key = np.zeros(cap, np.int64)
    beg = np.zeros(cap, np.int32)
    end = np.zeros(cap, np.int32)
    rev = np.zeros(cap, np.uint8)
    rec = np.zeros(cap, np.uint32)
    st = C.c_int32(0)
    k = lib().or_summarize_ranges(pay.ctypes.data, off.ctypes.data, n, split_status, key.ctypes.data,
                                  beg.ctypes.data, end.ctypes.data, rev.ctypes.data, rec.ctypes.data,
                                  cap, C.byref(st))
    assert k >= 0, k
    return dict(key=key[:k], beg=beg[:k], end=end[:k], rev=rev[:k], record=rec[:k], status=st.value)


def name_order(payload, offsets):
    """FixMateMapper's shuffle order: (Text(readName), input order)."""
    pay, off, n = _pay(payload, offsets)
    perm = np.zeros(max(n, 1), np.uint32)
    lib().or_name_order(pay.ctypes.data, off.ctypes.data, n, perm.ctypes.data)
    return perm[:n]


def fixmate(payload, offsets):
    """FixMateReducer (FixMate.java:230-277) over the name-sorted records -> dict(payload,
    offsets, src, status)."""
    pay, off, n = _pay(payload, offsets)
    cap = 2 * n + 1
    pay_cap = 2 * int(off[-1]) + 16 * cap
    out = np.zeros(max(pay_cap, 1), np.uint8)
    ooff = np.zeros(cap + 1, np.uint64)
    src = np.zeros(cap, np.uint32)
    st = C.c_int32(0)
    k = lib().or_fixmate(pay.ctypes.data, off.ctypes.data, n, out.ctypes.data, ooff.ctypes.data,
                         src.ctypes.data, cap, pay_cap, C.byref(st))
    assert k >= 0, k
    return dict(payload=out[:int(ooff[k])], offsets=ooff[:k + 1], src=src[:k], status=st.value)


# ---- BCF: hbam_oracle_bcf.c -------------------------------------------------
def is_bgzf(data):
    """BlockCompressedInputStream.isValidFile: an 18-byte BGZF member header at offset 0."""
    b = bytes(data[:18])
    return (len(b) == 18 and b[:4] == b"\x1f\x8b\x08\x04" and b[10:12] == b"\x06\x00"
            and b[12:14] == b"BC" and b[14:16] == b"\x02\x00")


def bcf_stream_prefix(data, want=1 << 20):
    """Uncompressed stream bytes at the start of a (BGZF or plain) BCF file."""
    if not is_bgzf(data):
        return bytes(data[:want])
    out, p = [], 0
    n = 0
    while p + 18 <= len(data) and n < want:
        bl = int.from_bytes(bytes(data[p + 16:p + 18]), "little") + 1
        rc, u = inflate_block(bytes(data[p:p + bl]), check_crc=False)
        if rc:
            break
        out.append(u)
        n += len(u)
        p += bl
    return b"".join(out)


def bcf_header(data):
    """BCF2Codec.readHeader: dict(n_contig, n_sample, n_dict, header_len, bgzf) or an error code."""
    u = bcf_stream_prefix(data)
    a, p = _buf(u if u else b"\0")
    nc, ns, nd, hl = C.c_int32(), C.c_int32(), C.c_int32(), C.c_uint64()
    rc = lib().or_bcf_read_header(p, len(u), C.byref(nc), C.byref(ns), C.byref(nd), C.byref(hl))
    if rc:
        return rc
    return dict(n_contig=nc.value, n_sample=ns.value, n_dict=nd.value, header_len=hl.value,
                bgzf=is_bgzf(data))


def guess_bcf_record_start(data, beg, end, h):
    """BCFSplitGuesser.guessNextBCFRecordStart -> (guess, err)."""
    a, p = _buf(data)
    err = C.c_int(0)
    r = lib().or_guess_bcf_record_start(p, len(a), beg, end, int(h["bgzf"]), h["n_contig"],
                                        h["n_sample"], h["n_dict"], C.byref(err))
    return r, err.value


def read_bcf_split_ex(data, start, end_or_len, h, cap=1 << 20):
    """read_bcf_split with every record column (l_shared, l_indiv, rlen, qual, n_allele_info,
    n_fmt_sample) and each record's bytes (l_shared, l_indiv, site block, genotype block)."""
    a, p = _buf(data)
    cols = dict(rel=np.zeros(cap, np.int64), chrom=np.zeros(cap, np.int32), pos=np.zeros(cap, np.int32),
                key=np.zeros(cap, np.int64), l_shared=np.zeros(cap, np.int32), l_indiv=np.zeros(cap, np.int32),
                rlen=np.zeros(cap, np.int32), qual=np.zeros(cap, np.uint32), n_allele_info=np.zeros(cap, np.int32),
                n_fmt_sample=np.zeros(cap, np.int32))
    bcap = 2 * len(a) + (1 << 22)
    byts = np.zeros(bcap, np.uint8)
    boff = np.zeros(cap + 1, np.uint64)
    st = C.c_int(0)
    f = lib().or_read_bcf_split_ex
    f.restype = C.c_int64
    n = int(f(p, C.c_uint64(len(a)), C.c_int(int(h["bgzf"])), C.c_uint64(start), C.c_uint64(end_or_len),
              C.c_int32(h["n_contig"]), C.c_int32(h["n_sample"]), C.c_int32(h["n_dict"]),
              C.c_uint64(h["header_len"]), *[C.c_void_p(cols[k].ctypes.data) for k in
                                             ("rel", "chrom", "pos", "key", "l_shared", "l_indiv", "rlen", "qual",
                                              "n_allele_info", "n_fmt_sample")],
              C.c_void_p(byts.ctypes.data), C.c_uint64(bcap), C.c_void_p(boff.ctypes.data), C.c_uint64(cap),
              C.byref(st)))
    m = min(n, cap)
    out = {k: v[:m].copy() for k, v in cols.items()}
    out.update(n=n, status=st.value, bytes=byts[:int(boff[m])].tobytes(), boff=boff[:m + 1].copy())
    return out


def read_bcf_split(data, start, end_or_len, h, cap=1 << 22):
    """BCFRecordReader over one split: BGZF -> FileVirtualSplit [start, end_or_len) (virtual);
    uncompressed -> FileSplit start, length = end_or_len.  dict(n, status, rel, chrom, pos, key)."""
    a, p = _buf(data)
    rel = np.zeros(cap, np.int64)
    chrom = np.zeros(cap, np.int32)
    pos = np.zeros(cap, np.int32)
    key = np.zeros(cap, np.int64)
    st = C.c_int(0)
    n = lib().or_read_bcf_split(p, len(a), int(h["bgzf"]), start, end_or_len, h["n_contig"],
                                h["n_sample"], h["n_dict"], h["header_len"], rel.ctypes.data,
                                chrom.ctypes.data, pos.ctypes.data, key.ctypes.data, cap, C.byref(st))
    n = int(n)
    m = min(n, cap)
    return dict(n=n, status=st.value, rel=rel[:m].copy(), chrom=chrom[:m].copy(), pos=pos[:m].copy(),
                key=key[:m].copy())


def bcf_splits(data, split_size, h):
    """VCFInputFormat.addGuessedSplits for one BCF path (VCFInputFormat.java:241-310) over
    FileInputFormat's splits of split_size: list of (start, end) — virtual offsets for BGZF
    (FileVirtualSplit), (start, length) for uncompressed (FileSplit); or an error code
    (OR_EIO: "no records in first split", or the guesser's escaping exception)."""
    n = len(data)
    fs = []
    b = 0
    while n - b > 1.1 * split_size:  # FileInputFormat SPLIT_SLOP
        fs.append((b, split_size))
        b += split_size
    if n - b > 0:
        fs.append((b, n - b))
    out = []
    bg = bool(h["bgzf"])
    for beg, ln in fs:
        end = beg + ln
        g, err = guess_bcf_record_start(data, beg, end, h)
        if err:
            return err
        align_end = (end << 16 | 0xffff) if bg else end
        if g == end:
            if not out:
                return -1
            if bg:
                out[-1] = (out[-1][0], align_end)
                continue
            prev = out.pop()
            out.append((g, align_end - g))  # the reference's FileSplit(path, alignBeg, length)
            continue
        out.append((g, align_end) if bg else (g, align_end - g))
    return out
