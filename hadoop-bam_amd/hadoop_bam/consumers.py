"""Read-name / CIGAR keyed consumers of the BAM read path, host mirror of the
reference classes over the device entry points:

* Range, RangeCount, SummarizeRecordReader, SummarizeInputFormat
  (cli/plugins/chipster/Summarize.java:563-755): every mapped record's CIGAR as reference ranges
  keyed by getKey0(refIdx, centre of mass) — hbam_summarize_ranges per decoded window;
* FixMateMapper / FixMateReducer (cli/plugins/FixMate.java:209-277): the Text(readName) shuffle
  and the reducer's pairing + SamPairUtil.setMateInfo — hbam_name_order / hbam_fixmate over the
  records of the job's splits, gathered on the device.

No CPU fallback: the work runs in libhbam.so; without it _lib raises HbamUnavailable."""
import ctypes as C

import numpy as np

from . import _lib
from .formats import (BAMInputFormat, Configuration, LongWritable, WINDOW_BYTES_PROPERTY, context,
                      raise_for, read_header)


class IndexOutOfBoundsException(IndexError):
    pass


def _raise(code, msg):
    if code == _lib.HBAM_EINDEX:
        raise IndexOutOfBoundsException(msg)
    raise_for(code, msg)


class Range:
    """Summarize.java:563-589"""

    def __init__(self, b=0, e=0, rev=False):
        self.beg, self.end, self.reverseStrand = int(b), int(e), bool(rev)

    def getCentreOfMass(self):  # :575-577, long arithmetic, truncated to int
        s = self.beg + self.end
        q = abs(s) // 2 * (1 if s >= 0 else -1)
        q &= 0xffffffff
        return q - (1 << 32) if q >> 31 else q

    def __eq__(self, o):
        return (self.beg, self.end, self.reverseStrand) == (o.beg, o.end, o.reverseStrand)

    def __repr__(self):
        return "Range(%d, %d, %s)" % (self.beg, self.end, self.reverseStrand)


class RangeCount:
    """Summarize.java:591-623 (the reducer's output value; tabix-compatible toString)."""

    def __init__(self, rng=None, count=0, rid=0):
        self.range = rng or Range()
        self.count, self.rid = count, rid

    def __str__(self):
        return "%d\t%d\t%d\t%d" % (self.rid, self.range.beg, self.range.end, self.count)

    def compareTo(self, o):
        return (self.range.beg > o.range.beg) - (self.range.beg < o.range.beg)


class SummarizeRecordReader:
    """Summarize.java:664-755.  The base reader is the BAM read path itself: the split is decoded
    window by window on the device (hbam_split_open/next) and each window's records are cut into
    ranges on the device (hbam_summarize_ranges); nextKeyValue walks them and raises where the
    reference's nextKeyValue raises (the base reader's exception, IllegalArgumentException for a
    bad CIGAR op, IndexOutOfBoundsException for a record without a range)."""

    def __init__(self):
        self.key = LongWritable()
        self._gen = None

    def initialize(self, split, ctx=None):
        conf = ctx if isinstance(ctx, Configuration) else Configuration()
        path = split.getPath()
        data = path if isinstance(path, (bytes, bytearray, np.ndarray)) else np.memmap(path, np.uint8, "r")
        self.ctxt = context(conf)
        h = read_header(data, self.ctxt)
        if isinstance(h, int):
            raise_for(h, "cannot read SAM header")
        window = int(conf.get(WINDOW_BYTES_PROPERTY, 1 << 30))
        self._gen = self.ctxt.split_stream(data, split.getStartVirtualOffset(), split.getEndVirtualOffset(),
                                           h["n_ref"], window, host=False)
        self._r = None
        self._i = 0
        self._value = None
        self._done = False

    def _next_window(self):
        try:
            d = next(self._gen)
        except StopIteration:
            self._done = True
            return False
        self._r = self.ctxt.summarize_ranges(d)
        self._i = 0
        return True

    def nextKeyValue(self):
        while not self._done and (self._r is None or self._i >= len(self._r["key"])):
            if self._r is not None and self._r["status"] not in (0, _lib.HBAM_EMORE):
                st = self._r["status"]
                self._r = None
                self._done = True
                _raise(st, "SummarizeRecordReader.nextKeyValue")
            if not self._next_window():
                return False
        if self._done:
            return False
        i = self._i
        self._i += 1
        r = self._r
        self.key.set(int(r["key"][i]))
        self._value = Range(r["beg"][i], r["end"][i], r["rev"][i])
        return True

    def getCurrentKey(self):
        return self.key

    def getCurrentValue(self):
        return self._value

    def close(self):
        if self._gen is not None:
            self._gen.close()
        self._gen = None


class SummarizeInputFormat(BAMInputFormat):
    """Summarize.java:632-663: the splits of the BAM input format, records read as ranges."""

    def createRecordReader(self, split, ctx=None):
        rr = SummarizeRecordReader()
        rr.initialize(split, ctx)
        return rr


class Text:
    """org.apache.hadoop.io.Text over the read-name bytes."""

    def __init__(self, b=b""):
        self.bytes = bytes(b)

    def __eq__(self, o):
        return self.bytes == o.bytes

    def __repr__(self):
        return "Text(%r)" % self.bytes


def fix_mate(splits, conf=None):
    """FixMate's job body (FixMate.java:145-190, no combiner, no global sort): the records of every
    split (BAMRecordReader over each FileVirtualSplit) through FixMateMapper's Text(readName) key,
    the shuffle and FixMateReducer.  Returns (keys, payloads, offsets): the reducer's writes in
    output order as Text keys and SAMRecordWritable payload bytes.  All record work runs on the
    device: each split is decoded and packed (hbam_decode_split + hbam_gather_records) into one
    buffer, then hbam_fixmate orders, groups, pairs and re-encodes."""
    import torch
    conf = conf or Configuration()
    ctx = context(conf)
    L = ctx.L
    parts, sizes = [], []
    for sp in splits:
        path = sp.getPath()
        data = path if isinstance(path, (bytes, bytearray, np.ndarray)) else np.memmap(path, np.uint8, "r")
        h = read_header(data, ctx)
        if isinstance(h, int):
            raise_for(h, "cannot read SAM header")
        rc, d = ctx.decode_split_device(data, sp.getStartVirtualOffset(), sp.getEndVirtualOffset(), h["n_ref"])
        if rc:
            raise_for(rc, ctx.last_error())
        n = int(d.n_records)
        ub, ro, bs = (C.cast(x, C.c_void_p) for x in (d.ubuf, d.rec_off, d.block_size))
        off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()  # the library's stream does not order after torch's
        tot = C.c_uint64(0)
        rc = L.hbam_gather_records(ctx.h, ub, ro, bs, None, n, None, 0,
                                   C.c_void_p(off.data_ptr()), C.byref(tot))
        if rc:
            raise RuntimeError("hbam_gather_records: %s" % ctx.last_error())
        pay = torch.empty(max(int(tot.value), 1), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        rc = L.hbam_gather_records(ctx.h, ub, ro, bs, None, n, C.c_void_p(pay.data_ptr()), int(tot.value), C.c_void_p(off.data_ptr()),
                                   C.byref(tot))
        if rc:
            raise RuntimeError("hbam_gather_records: %s" % ctx.last_error())
        parts.append((pay[:int(tot.value)], off[:-1]))
        sizes.append(int(tot.value))
        if d.status not in (0,):
            raise_for(int(d.status), "BAMRecordReader.nextKeyValue")
    base = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    pay = torch.cat([p for p, _ in parts]) if parts else torch.zeros(1, dtype=torch.uint8, device="cuda")
    rec_off = (torch.cat([o + int(base[i]) for i, (_, o) in enumerate(parts)]) if parts
               else torch.zeros(1, dtype=torch.int64, device="cuda"))
    torch.cuda.synchronize()
    n = int(rec_off.numel()) if parts else 0
    r = ctx.fixmate(pay.data_ptr(), rec_off.data_ptr(), n)
    if r["status"]:
        raise_for(r["status"], "FixMateReducer: setMateInfo on an unparsable record")
    out_off = r["offsets"].astype(np.int64)
    keys = []
    for k in range(len(r["src"])):
        p = r["payload"][out_off[k]:out_off[k + 1]]
        lrn = int(p[12])
        keys.append(Text(bytes(p[36:36 + max(lrn - 1, 0)])))
    return keys, r["payload"], out_off
