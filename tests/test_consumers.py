"""Read-name / CIGAR keyed consumers: SummarizeRecordReader's ranges
(cli/plugins/chipster/Summarize.java:664-755) and FixMate's name shuffle + reducer
(cli/plugins/FixMate.java:209-277).

CPU tests pin the oracle (oracle/hbam_oracle_f4.c) against an independent pure-Python reading of
the same Java lines; GPU tests require the HIP path (hbam_summarize_ranges / hbam_name_order /
hbam_fixmate through the C ABI) to equal the oracle bit for bit."""
import ctypes as C
import os

import numpy as np
import pytest

import f4_records as F
from conftest import ROOT


def _i32(x):
    x &= 0xffffffff
    return x - (1 << 32) if x >> 31 else x


def _i64(x):
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >> 63 else x


def _fields(rec):
    import struct
    bs, ref, pos, lrn, mapq, bin_, nc, flag, lseq, nref, npos, tlen = struct.unpack_from("<iiiBBHHHiiii", rec)
    # a CIGAR past the record's block_size: getCigar's lazy read throws (None here)
    cig = struct.unpack_from("<%dI" % nc, rec, 36 + lrn) if 32 + lrn + 4 * nc <= bs else None
    return dict(ref=ref, pos=pos, lrn=lrn, flag=flag, cigar=cig, name=bytes(rec[36:36 + max(lrn - 1, 0)]))


def py_summarize(recs):
    """Summarize.java:693-755, read line by line (Java int wrap, long centre of mass)."""
    out, status = [], 0
    for i, rec in enumerate(recs):
        f = _fields(rec)
        start = _i32(f["pos"] + 1)
        if (f["flag"] & 4) or f["ref"] < 0 or start < 0:
            continue
        if f["cigar"] is None:
            return out, -3
        ranges = []
        b = e = start
        for c in f["cigar"]:
            op, ln = c & 15, c >> 4
            if op > 8:
                return out, -6
            if op in (0, 7, 8):
                e = _i32(e + ln)
                continue
            if b != e:
                ranges.append((b, _i32(e - 1)))
                b = e
            if op in (2, 3):
                b = _i32(b + ln)
                e = b
        if b != e:
            ranges.append((b, _i32(e - 1)))
        if not ranges:
            return out, -13
        key = None
        for (rb, re_) in ranges:
            s = rb + re_
            com = _i32(int(abs(s) // 2) * (1 if s >= 0 else -1))  # Java long division truncates
            if key is None:
                key = _i64((f["ref"] << 32) | (com & 0xffffffffffffffff if com < 0 else com))
            else:
                key = _i64(((key & ((1 << 64) - 1)) >> 32 << 32) | (com & ((1 << 64) - 1)))
            out.append((key, rb, re_, 1 if f["flag"] & 0x10 else 0, i))
    return out, status


def _oracle():
    import oracle
    return oracle


def test_summarize_known_answer():
    """5S10M3I10M2D5M4N6M2H at 1-based 100, reverse: (100,109) (110,119) (122,126) (131,136)."""
    o = _oracle()
    pay, off = F.pack([F.summarize_edge_records()[0]])
    r = o.summarize_ranges(pay, off)
    assert r["status"] == 0
    assert list(zip(r["beg"], r["end"])) == [(100, 109), (110, 119), (122, 126), (131, 136)]
    assert list(r["rev"]) == [1, 1, 1, 1]
    assert list(r["key"]) == [(3 << 32) | 104, (3 << 32) | 114, (3 << 32) | 124, (3 << 32) | 133]


@pytest.mark.parametrize("kind", [None, "op", "empty", "overrun"])
def test_summarize_oracle_vs_java_reading(kind):
    o = _oracle()
    recs = F.summarize_edge_records() if kind is None else F.summarize_error_records(kind)
    want, wst = py_summarize(recs)
    pay, off = F.pack(recs)
    r = o.summarize_ranges(pay, off)
    got = list(zip(r["key"].tolist(), r["beg"].tolist(), r["end"].tolist(), r["rev"].tolist(),
                   r["record"].tolist()))
    assert got == want
    assert r["status"] == wst


def test_name_order_matches_text_order():
    o = _oracle()
    recs = F.names_records()
    pay, off = F.pack(recs)
    perm = o.name_order(pay, off)
    names = [_fields(r)["name"] for r in recs]
    assert perm.tolist() == sorted(range(len(recs)), key=lambda i: (names[i], i))


def py_reduce_plan(recs):
    """FixMateReducer.reduce's writes (FixMate.java:241-276) as (src, mate) over the shuffle."""
    names = [_fields(r)["name"] for r in recs]
    order = sorted(range(len(recs)), key=lambda i: (names[i], i))
    sec = [bool(_fields(r)["flag"] & 0x100) for r in recs]
    out, g = [], 0
    while g < len(order):
        ge = g
        while ge < len(order) and names[order[ge]] == names[order[g]]:
            ge += 1
        it = iter(order[g:ge])
        vals = list(order[g:ge])
        k = 0
        while k < len(vals):
            a = vals[k]
            k += 1
            if sec[a]:
                out.append((a, None))
                continue
            b = None
            while k < len(vals):
                b = vals[k]
                k += 1
                if not sec[b]:
                    break
                out.append((b, None))
            if b is None:
                out.append((a, None))
                break
            out.append((a, b))
            out.append((b, a))
        g = ge
    return out


def test_fixmate_plan_and_quirk():
    o = _oracle()
    recs = F.fixmate_records()
    pay, off = F.pack(recs)
    r = o.fixmate(pay, off)
    assert r["status"] == 0
    plan = py_reduce_plan(recs)
    assert r["src"].tolist() == [s for s, _ in plan]
    # the quirk: a group "PSS" writes S, S, then P and the last S mated -> that S twice
    names = [_fields(x)["name"] for x in recs]
    from collections import Counter
    dup = Counter(r["src"].tolist())
    twice = [i for i, c in dup.items() if c == 2]
    assert twice and all(_fields(recs[i])["flag"] & 0x100 for i in twice)
    # untouched writes are the input bytes
    for k, (s, m) in enumerate(plan):
        got = bytes(r["payload"][int(r["offsets"][k]):int(r["offsets"][k + 1])])
        if m is None:
            assert got == bytes(recs[s])


def test_fixmate_mate_fields():
    """setMateInfo on a both-mapped pair: mate ref/pos/strand from the other record, MQ = the
    other's MAPQ (in place), MC removed, TLEN = 5'(b) - 5'(a) +/- 1 with opposite signs."""
    import struct
    o = _oracle()
    a = F.record(b"q", flag=0x41, ref=2, pos=100, mapq=30, cigar=((50, 0),), l_seq=50,
                 aux=F.aux_z("MC", "9M") + F.aux_int("MQ", "C", 200) + F.aux_int("NM", "i", 2))
    b = F.record(b"q", flag=0x91, ref=2, pos=300, mapq=200, cigar=((40, 0), (10, 2)), l_seq=40)
    pay, off = F.pack([a, b])
    r = o.fixmate(pay, off)
    ra = bytes(r["payload"][int(r["offsets"][0]):int(r["offsets"][1])])
    rb = bytes(r["payload"][int(r["offsets"][1]):int(r["offsets"][2])])
    fa, fb = struct.unpack_from("<iiiBBHHHiiii", ra), struct.unpack_from("<iiiBBHHHiiii", rb)
    # a: mate = b (ref 2, pos 300, reverse) ; 5' of b = end = 301 + 50 - 1 = 350 ; 5' of a = 101
    assert fa[9:12] == (2, 300, 350 - 101 + 1)
    assert fa[7] & 0x20 and not fa[7] & 0x8
    assert fb[9:12] == (2, 100, -(350 - 101 + 1))
    assert not fb[7] & 0x20
    assert ra.endswith(b"MQc\x00" + b"NMc\x02") or b"MQC\xc8" in ra  # MQ = 200 -> 'C', in place
    assert b"MC" not in ra[36:]
    assert rb.endswith(b"MQc\x1e")  # appended: MAPQ 30 -> 'c'


# ---- HIP path through the C ABI ------------------------------------------------------------
def _ctx():
    import torch  # torch's HIP runtime must open the device before libhbam's (_lib.Context)
    torch.cuda.init()
    from hadoop_bam import _lib
    return _lib.Context(0)


def _dev_records(recs_or_pay, off=None):
    import torch
    if off is None:
        pay, off = F.pack(recs_or_pay)
    else:
        pay = recs_or_pay
    tp = torch.from_numpy(np.ascontiguousarray(pay)).cuda()
    to = torch.from_numpy(np.ascontiguousarray(off).view(np.int64)).cuda()
    torch.cuda.synchronize()
    return tp, to, len(off) - 1


def _fake_columns(tp, to, n, status=0):
    from hadoop_bam import _lib
    d = _lib.Columns()
    d.n_records = n
    d.status = status
    d.ubuf = C.cast(C.c_void_p(tp.data_ptr()), _lib._u8p)
    d.rec_off = C.cast(C.c_void_p(to.data_ptr()), _lib._u64p)
    return d


def _same_ranges(got, want):
    for k in ("key", "beg", "end", "rev", "record"):
        assert np.array_equal(got[k], want[k]), k
    assert got["status"] == want["status"]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [None, "op", "empty", "overrun"])
def test_summarize_device_edges(kind):
    recs = F.summarize_edge_records() if kind is None else F.summarize_error_records(kind)
    ctx = _ctx()
    tp, to, n = _dev_records(recs)
    got = ctx.summarize_ranges(_fake_columns(tp, to, n))
    pay, off = F.pack(recs)
    _same_ranges(got, _oracle().summarize_ranges(pay, off))


GOLDEN = [f for f in ("small_pe.bam", "edge_uniform_long.bam", "edge_unsorted_l1.bam")]


@pytest.mark.gpu
@pytest.mark.parametrize("name", GOLDEN)
def test_summarize_device_on_decoded_split(name):
    o = _oracle()
    data = np.fromfile(os.path.join(ROOT, "tests", "golden", name), np.uint8)
    h = o.read_header(data)
    v_end = (len(data) << 16) | 0xffff
    ref = o.read_split(data, h["first_voffset"], v_end)
    pay, off = o.record_payloads(ref)
    want = o.summarize_ranges(pay, off, ref["status"])
    ctx = _ctx()
    rc, d = ctx.decode_split_device(data, h["first_voffset"], v_end, h["n_ref"])
    assert rc == 0
    assert int(d.n_records) == ref["n"]
    got = ctx.summarize_ranges(d)
    assert len(got["key"]) > 0
    _same_ranges(got, want)


@pytest.mark.gpu
def test_name_order_device():
    recs = F.names_records(n=3000, seed=12)
    import torch
    ctx = _ctx()
    tp, to, n = _dev_records(recs)
    perm = torch.zeros(n, dtype=torch.int32, device="cuda")
    ctx.name_order(tp.data_ptr(), to.data_ptr(), n, perm.data_ptr())
    pay, off = F.pack(recs)
    assert perm.cpu().numpy().view(np.uint32).tolist() == _oracle().name_order(pay, off).tolist()


def _same_fixmate(got, want):
    assert got["status"] == want["status"]
    assert np.array_equal(got["src"], want["src"])
    assert np.array_equal(got["offsets"], want["offsets"])
    assert np.array_equal(got["payload"], want["payload"])


@pytest.mark.gpu
@pytest.mark.parametrize("copies", [1, 60])
def test_fixmate_device_edges(copies):
    recs = []
    for c in range(copies):  # copies share names: key groups of up to 4 * copies records
        recs += F.fixmate_records(seed=5 + c)
    ctx = _ctx()
    tp, to, n = _dev_records(recs)
    got = ctx.fixmate(tp.data_ptr(), to.data_ptr(), n)
    pay, off = F.pack(recs)
    _same_fixmate(got, _oracle().fixmate(pay, off))


@pytest.mark.gpu
def test_fixmate_device_malformed_aux():
    """A mated record whose attributes do not parse: the job fails at that write (SAMFormatException)."""
    recs = F.fixmate_records()[:40]
    bad = F.record(b"zzz", flag=0x41, ref=0, pos=5, aux=b"NMq\x01")  # unknown type 'q'
    mate = F.record(b"zzz", flag=0x81, ref=0, pos=9)
    recs = recs + [bad, mate]
    ctx = _ctx()
    tp, to, n = _dev_records(recs)
    got = ctx.fixmate(tp.data_ptr(), to.data_ptr(), n)
    pay, off = F.pack(recs)
    want = _oracle().fixmate(pay, off)
    assert want["status"] == -3
    _same_fixmate(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("field", ["cigar", "seq"])
def test_fixmate_device_layout_overrun(field):
    """A record whose n_cigar / l_seq claims more bytes than its block_size holds (a decoded
    split hands such a record out with status OK, layout_ok 0): the device never reads past the
    record, and the job fails before any output as the oracle's (SAMFormatException)."""
    recs = F.fixmate_records()[:40]
    recs.insert(17, F.overrun_record(field))
    ctx = _ctx()
    tp, to, n = _dev_records(recs)
    got = ctx.fixmate(tp.data_ptr(), to.data_ptr(), n)
    pay, off = F.pack(recs)
    want = _oracle().fixmate(pay, off)
    assert want["status"] == -3 and len(want["src"]) == 0
    _same_fixmate(got, want)


@pytest.mark.gpu
def test_fixmate_device_on_decoded_split():
    o = _oracle()
    data = np.fromfile(os.path.join(ROOT, "tests", "golden", "small_pe.bam"), np.uint8)
    h = o.read_header(data)
    v_end = (len(data) << 16) | 0xffff
    ref = o.read_split(data, h["first_voffset"], v_end)
    pay, off = o.record_payloads(ref)
    want = o.fixmate(pay, off)
    ctx = _ctx()
    rc, d = ctx.decode_split_device(data, h["first_voffset"], v_end, h["n_ref"])
    assert rc == 0
    ub = C.cast(d.ubuf, C.c_void_p).value
    ro = C.cast(d.rec_off, C.c_void_p).value
    got = ctx.fixmate(ub, ro, int(d.n_records))
    assert got["n_groups"] == len(set(bytes(want["payload"][int(want["offsets"][k]) + 36:
                                                           int(want["offsets"][k]) + 35 +
                                                           int(want["payload"][int(want["offsets"][k]) + 12])])
                                      for k in range(len(want["src"]))))
    _same_fixmate(got, want)


# ---- the mirror classes (host side of the drop-in) -----------------------------------------
def _golden_splits(name, split_size):
    from hadoop_bam import formats
    o = _oracle()
    data = np.fromfile(os.path.join(ROOT, "tests", "golden", name), np.uint8)
    beg, end = o.file_splits(len(data), split_size)
    vs, ve = o.probabilistic_splits(data, beg, end)
    return data, [formats.FileVirtualSplit(data, int(a), int(b)) for a, b in zip(vs, ve)]


@pytest.mark.gpu
def test_summarize_record_reader_mirror():
    from hadoop_bam import consumers, formats
    o = _oracle()
    data, splits = _golden_splits("small_pe.bam", 400_000)
    assert len(splits) >= 3
    conf = formats.Configuration({formats.WINDOW_BYTES_PROPERTY: 300_000})
    for sp in splits:
        ref = o.read_split(data, sp.getStartVirtualOffset(), sp.getEndVirtualOffset())
        pay, off = o.record_payloads(ref)
        want = o.summarize_ranges(pay, off, ref["status"])
        rr = consumers.SummarizeInputFormat().createRecordReader(sp, conf)
        keys, rngs = [], []
        raised = 0
        try:
            while rr.nextKeyValue():
                keys.append(rr.getCurrentKey().get())
                v = rr.getCurrentValue()
                rngs.append((v.beg, v.end, int(v.reverseStrand)))
        except consumers.IndexOutOfBoundsException:
            raised = -13
        except formats.IllegalArgumentException:
            raised = -6
        except formats.SAMFormatException:
            raised = -3
        rr.close()
        assert raised == want["status"]
        assert keys == want["key"].tolist()
        assert rngs == list(zip(want["beg"].tolist(), want["end"].tolist(), want["rev"].tolist()))


@pytest.mark.gpu
def test_fix_mate_job_mirror():
    from hadoop_bam import consumers
    o = _oracle()
    data, splits = _golden_splits("small_pe.bam", 400_000)
    pays, offs, base = [], [], 0
    for sp in splits:
        ref = o.read_split(data, sp.getStartVirtualOffset(), sp.getEndVirtualOffset())
        p, f = o.record_payloads(ref)
        pays.append(p)
        offs.append(f[:-1].astype(np.uint64) + np.uint64(base))
        base += len(p)
    pay = np.concatenate(pays)
    off = np.concatenate(offs + [np.array([base], np.uint64)])
    want = o.fixmate(pay, off)
    keys, got_pay, got_off = consumers.fix_mate(splits)
    assert np.array_equal(got_off.astype(np.uint64), want["offsets"])
    assert np.array_equal(got_pay, want["payload"])
    names = [bytes(want["payload"][int(want["offsets"][k]) + 36:int(want["offsets"][k]) + 36 +
                   int(want["payload"][int(want["offsets"][k]) + 12]) - 1]) for k in range(len(keys))]
    assert [k.bytes for k in keys] == names
