"""Host-side mirror of Hadoop-BAM's BCF input classes over the MI355X C ABI.

BCFSplitGuesser (BCFSplitGuesser.java:52-455), BCFRecordReader (BCFRecordReader.java:52-175) and
the BCF half of VCFInputFormat (VCFInputFormat.java:197-310), same names, argument meaning and
exceptions.  The BGZF blocks, the guesses and the record decode run in libhbam.so
(hbam_bcf.hip); the record decode restates a subset of htsjdk's BCF2Codec (parity unpinned,
oracle/hbam_oracle_bcf.c).
"""
import struct

import numpy as np

from . import _lib
from .formats import (FileSplit, FileVirtualSplit, IOException, SeekableFile, compute_file_splits,
                      context, raise_for)


class TribbleException(RuntimeError):
    """htsjdk.tribble.TribbleException (BCF2Codec's error for unreadable records)."""


class BCFDecodeRuntimeException(RuntimeError):
    """Another RuntimeException out of BCF2Codec.decode (IndexOutOfBounds, NPE, ClassCast)."""


def _raise(code, msg=""):
    if code == _lib.HBAM_ETRIBBLE:
        raise TribbleException(msg or "TribbleException")
    if code == _lib.HBAM_ERUNTIME:
        raise BCFDecodeRuntimeException(msg or "RuntimeException")
    raise_for(code, msg)


def is_bgzf(head):
    """BlockCompressedInputStream.isValidFile: a BGZF member header at offset 0."""
    b = bytes(head[:18])
    return (len(b) == 18 and b[:4] == b"\x1f\x8b\x08\x04" and b[10:12] == b"\x06\x00"
            and b[12:14] == b"BC" and b[14:16] == b"\x02\x00")


def read_bcf_header(ss, ctx):
    """BCF2Codec.readHeader over a growing prefix of the stream -> header dict."""
    n = min(ss.length, 1 << 20)
    while True:
        h = ctx.bcf_parse_header(ss.read_at(0, n))
        if isinstance(h, dict) or h != _lib.HBAM_EMORE or n >= ss.length:
            if isinstance(h, int):
                _raise(h, "cannot read the BCF header")
            return h
        n = min(ss.length, 4 * n)


class BCFSplitGuesser:
    """BCFSplitGuesser.java:52-455: a guess reads only its window (hbam_guess_bcf_window_len
    bytes at beg, :133-145) and runs on the device (k_guess_bcf)."""

    def __init__(self, ss, header_stream=None, conf=None):
        self.ss = SeekableFile(ss)
        self.ctx = context(conf)
        self.h = read_bcf_header(self.ss if header_stream is None else SeekableFile(header_stream), self.ctx)
        self.h["bgzf"] = is_bgzf(self.ss.read_at(0, 18))  # :99-103: the data stream decides

    def isBGZF(self):
        return bool(self.h["bgzf"])

    def guessNextBCFRecordStart(self, beg, end):
        wl = self.ctx.guess_bcf_window_len(self.ss.length, beg, end, self.isBGZF())
        w = self.ss.read_at(beg, wl)
        rc, out, err = self.ctx.guess_bcf_windows(w, [0, wl], self.ss.length, [beg], [end], self.h)
        raise_for(rc, self.ctx.last_error())
        _raise(int(err[0]), "exception escaped the guesser")
        return int(out[0])


class BCFRecord:
    """The decoded fields of one BCF record (what VariantContextWritable exposes through
    VariantContext for the key: getChr / getStart) and its raw BCF2 bytes."""

    def __init__(self, cols, i):
        self._c, self._i = cols, i

    def getContigIndex(self):
        return int(self._c["chrom"][self._i])

    def getStart(self):  # 1-based
        return int(self._c["pos"][self._i]) + 1

    def getEnd(self):
        return self.getStart() + int(self._c["rlen"][self._i]) - 1

    def getNAlleles(self):
        return int(self._c["n_allele_info"][self._i]) >> 16

    def getNSamples(self):
        return int(self._c["n_fmt_sample"][self._i]) & 0xfffff

    def getQual(self):
        return struct.unpack("<f", struct.pack("<I", int(self._c["qual"][self._i])))[0]

    def toBCFBytes(self):
        if "data" not in self._c:
            raise ValueError("record bytes not kept")
        o = int(self._c["rec_off"][self._i])
        n = 8 + int(self._c["l_shared"][self._i]) + int(self._c["l_indiv"][self._i])
        return bytes(self._c["data"][o:o + n])


BCF_WINDOW_TAIL = 1 << 20  # compressed bytes read past vEnd's block offset at first


class BCFRecordReader:
    """BCFRecordReader.java:52-175.  FileVirtualSplit (BGZF, read through BGZFLimitingStream
    :177-237) or FileSplit (uncompressed); key = contig index << 32 | (start - 1)."""

    def __init__(self, keep_bytes=False):
        self.keep = keep_bytes
        self.cols = None

    def initialize(self, split, conf=None, data=None):
        ctx = context(conf)
        path = split.getPath()
        ss = SeekableFile(data if data is not None else path)
        h = read_bcf_header(ss, ctx)
        if isinstance(split, FileVirtualSplit):
            if not h["bgzf"]:
                raise IOException("FileVirtualSplit over an uncompressed BCF file")
            base = split.getStartVirtualOffset() >> 16
            start, end = split.getStartVirtualOffset(), split.getEndVirtualOffset()
        else:
            base = min(max(split.getStart(), h["header_len"]), ss.length)
            start, end = split.getStart(), split.getLength()
        # BGZF: the split's own bytes to past vEnd's block, longer only while BGZFLimitingStream
        # runs past the window (HBAM_EMORE: it stops only in a block starting exactly at vEnd's
        # offset, :206); uncompressed: to the end of the file (the reader's bound is a length)
        tail = BCF_WINDOW_TAIL
        while True:
            stop = ss.length if not h["bgzf"] else min(ss.length, (end >> 16) + tail)
            window = ss.read_at(base, stop - base)
            cols = ctx.bcf_decode_split(window, h, start, end, comp_base=base, file_len=ss.length,
                                        keep_data=self.keep)
            if cols["rc"]:
                raise_for(cols["rc"], cols.get("error", ""))
            if cols["status"] != _lib.HBAM_EMORE or stop == ss.length:
                break
            tail *= 4
        self.window_bytes = stop - base
        self.cols, self.i = cols, -1
        self.key = None

    def nextKeyValue(self):
        c = self.cols
        if self.i + 1 < c["n"]:
            self.i += 1
            self.key = int(c["key"][self.i])
            return True
        self.i = c["n"]
        _raise(c["status"], "BCF2Codec.decode")
        return False

    def getCurrentKey(self):
        return self.key

    def getCurrentValue(self):
        return BCFRecord(self.cols, self.i)

    def close(self):
        self.cols = None


class VCFInputFormat:
    """The BCF half of VCFInputFormat.java:197-310: FileInputFormat splits of each BCF path are
    re-aligned to records by the guesser (addGuessedSplits :248-310)."""

    def getSplits(self, path, split_size, conf=None, data=None):
        ss = SeekableFile(data if data is not None else path)
        g = BCFSplitGuesser(ss, conf=conf)
        bg = g.isBGZF()
        out = []
        for fs in compute_file_splits(path, ss.length, split_size):
            beg, end = fs.getStart(), fs.getStart() + fs.getLength()
            align_beg = g.guessNextBCFRecordStart(beg, end)
            align_end = (end << 16 | 0xffff) if bg else end
            if align_beg == end:
                if not out:
                    raise IOException("'%s': no records in first split: bad BCF file or tiny split size?" % path)
                if bg:
                    out[-1].setEndVirtualOffset(align_end)
                    continue
                out.pop()
                out.append(FileSplit(path, align_beg, align_end - align_beg, fs.getLocations()))
                continue
            out.append(FileVirtualSplit(path, align_beg, align_end, fs.getLocations()) if bg
                       else FileSplit(path, align_beg, align_end - align_beg, fs.getLocations()))
        return out

    def createRecordReader(self, split, conf=None, data=None):
        rr = BCFRecordReader()
        rr.initialize(split, conf, data)
        return rr


def record_keys(reader):
    """All keys a reader hands out (and the exception it ends with) -> (np.int64 array, exc)."""
    keys = []
    try:
        while reader.nextKeyValue():
            keys.append(reader.getCurrentKey())
    except Exception as e:  # noqa: BLE001 - the exception is the result
        return np.array(keys, np.int64), e
    return np.array(keys, np.int64), None
