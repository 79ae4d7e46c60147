"""Host-side mirror of Hadoop-BAM's BAM input API over the MI355X C ABI.

Same class names, argument meaning and error behaviour as the reference's
org.seqdoop.hadoop_bam classes (file:line cited per class); the compute runs in
libhbam.so on the GPU.  The Java shim in java/ binds the same C ABI.
"""
import io
import os
import struct

import numpy as np

from . import _lib


# ---- exceptions (the Java classes the reference raises) ------------------------------
class IOException(Exception):
    pass


class SAMFormatException(RuntimeError):
    pass


class FileTruncatedException(RuntimeError):
    pass


class RuntimeIOException(RuntimeError):
    pass


class RuntimeEOFException(RuntimeError):
    pass


class IllegalArgumentException(ValueError):
    pass


class JavaRuntimeException(RuntimeError):
    """RuntimeException wrapping java.util.zip.DataFormatException."""


class NullPointerException(RuntimeError):
    pass


class ClassCastException(TypeError):
    pass


_EXC = {
    _lib.HBAM_EIO: IOException, _lib.HBAM_ETRUNC: FileTruncatedException,
    _lib.HBAM_EFORMAT: SAMFormatException, _lib.HBAM_ERUNTIMEIO: RuntimeIOException,
    _lib.HBAM_EEOF: RuntimeEOFException, _lib.HBAM_EREFID: IllegalArgumentException,
    _lib.HBAM_EDATA: JavaRuntimeException, _lib.HBAM_ENULL: NullPointerException,
    _lib.HBAM_ECLASSCAST: ClassCastException,
}


def raise_for(code, msg=""):
    if code == _lib.HBAM_OK:
        return
    exc = _EXC.get(code)
    if exc is None:
        raise _lib.HbamUnavailable("%s: %s" % (_lib.CODE_NAMES.get(code, code), msg))
    raise exc(msg or _lib.CODE_NAMES.get(code, str(code)))


# ---- Hadoop plumbing stand-ins ------------------------------------------------------
class Configuration(dict):
    """org.apache.hadoop.conf.Configuration (string properties)."""

    def get(self, k, default=None):
        return super().get(k, default)

    def getInt(self, k, default):
        v = self.get(k)
        return int(v) if v is not None else default


VALIDATION_STRINGENCY_PROPERTY = "hadoopbam.samheaderreader.validation-stringency"
CHECK_CRC_PROPERTY = "hadoopbam.hip.check-crc"
DEVICE_PROPERTY = "hadoopbam.hip.device"


class FileSplit:
    """org.apache.hadoop.mapreduce.lib.input.FileSplit."""

    def __init__(self, path, start, length, hosts=()):
        self.path, self.start, self.length, self.hosts = path, int(start), int(length), list(hosts)

    def getPath(self):
        return self.path

    def getStart(self):
        return self.start

    def getLength(self):
        return self.length

    def getLocations(self):
        return self.hosts


def compute_file_splits(path, file_len, split_size):
    """Hadoop 1.2.1 FileInputFormat.getSplits for one file (SPLIT_SLOP = 1.1)."""
    out, rem = [], file_len
    while split_size > 0 and rem / split_size > 1.1:
        out.append(FileSplit(path, file_len - rem, split_size))
        rem -= split_size
    if rem:
        out.append(FileSplit(path, file_len - rem, rem))
    return out


class FileVirtualSplit:
    """FileVirtualSplit.java:38-92 — a split in BGZF virtual offsets."""

    def __init__(self, path=None, v_start=0, v_end=0, locations=()):
        self.file, self.vStart, self.vEnd = path, int(v_start), int(v_end)
        self.locations = list(locations)

    def getLocations(self):
        return self.locations

    def getLength(self):  # :64-69
        vs_hi = self.vStart & ~0xffff
        ve_hi = self.vEnd & ~0xffff
        hi = ve_hi - vs_hi
        return (self.vEnd & 0xffff) - (self.vStart & 0xffff) if hi == 0 else hi

    def getPath(self):
        return self.file

    def getStartVirtualOffset(self):
        return self.vStart

    def getEndVirtualOffset(self):
        return self.vEnd

    def setStartVirtualOffset(self, vo):
        self.vStart = int(vo)

    def setEndVirtualOffset(self, vo):
        self.vEnd = int(vo)

    def write(self, out):  # :82-86  Text.writeString + two longs (big-endian)
        b = str(self.file).encode()
        out.write(_vlong(len(b)) + b + struct.pack(">qq", self.vStart, self.vEnd))

    def readFields(self, inp):  # :87-91
        n = _read_vlong(inp)
        self.file = inp.read(n).decode()
        self.vStart, self.vEnd = struct.unpack(">qq", inp.read(16))

    def __eq__(self, o):
        return (isinstance(o, FileVirtualSplit) and self.file == o.file and
                self.vStart == o.vStart and self.vEnd == o.vEnd)

    def __repr__(self):
        return "FileVirtualSplit(%s, %#x, %#x)" % (self.file, self.vStart, self.vEnd)


def _vlong(i):
    """Hadoop WritableUtils.writeVLong."""
    if -112 <= i <= 127:
        return struct.pack("b", i)
    ln = -112
    if i < 0:
        i ^= -1
        ln = -120
    tmp = i
    while tmp != 0:
        tmp >>= 8
        ln -= 1
    out = struct.pack("b", ln)
    n = -(ln + 120) if ln < -120 else -(ln + 112)
    for idx in range(n, 0, -1):
        out += struct.pack("B", (i >> ((idx - 1) * 8)) & 0xff)
    return out


def _read_vlong(inp):
    first = struct.unpack("b", inp.read(1))[0]
    if first >= -112:
        return first
    neg = first < -120
    n = -(first + 120) if neg else -(first + 112)
    i = 0
    for _ in range(n):
        i = (i << 8) | inp.read(1)[0]
    return i ^ -1 if neg else i


# ---- device file handles -------------------------------------------------------------
_CTX = {}


def context(conf=None):
    """One hbam context per (device, crc) in this process (one per Hadoop task thread)."""
    conf = conf or Configuration()
    dev = int(conf.get(DEVICE_PROPERTY, os.environ.get("LOCAL_RANK", 0)))
    crc = str(conf.get(CHECK_CRC_PROPERTY, "false")).lower() == "true"
    key = (dev, crc)
    if key not in _CTX:
        _CTX[key] = _lib.Context(dev, check_crc=crc, validate_refs=True)
    return _CTX[key]


def _read_file(path):
    if isinstance(path, (bytes, bytearray, np.ndarray)):
        return path
    with open(path, "rb") as f:
        return f.read()


class SeekableFile:
    """SeekableStream over a path, an open binary file or an in-memory buffer: only the byte
    ranges asked for are read (a guess reads its window, getSplits its FileSplits' windows and
    the header prefix — never the whole file)."""

    def __init__(self, src):
        self._f, self._own, self._buf = None, False, None
        if isinstance(src, SeekableFile):
            self._f, self._buf, self.length = src._f, src._buf, src.length
        elif isinstance(src, (bytes, bytearray, memoryview, np.ndarray)):
            self._buf = np.frombuffer(src, np.uint8) if not isinstance(src, np.ndarray) else src
            self.length = len(self._buf)
        elif hasattr(src, "read") and hasattr(src, "seek"):
            self._f = src
            self.length = src.seek(0, os.SEEK_END)
        else:
            self._f = open(src, "rb")
            self._own = True
            self.length = os.path.getsize(src)

    def read_at(self, off, n):
        n = max(0, min(int(n), self.length - int(off)))
        if n == 0:
            return b""
        if self._buf is not None:
            return bytes(self._buf[off:off + n])
        self._f.seek(off)
        return self._f.read(n)

    def close(self):
        if self._own and self._f is not None:
            self._f.close()
        self._f = None


def read_header_prefix(ss, ctx):
    """SAMHeaderReader.readSAMHeaderFrom over a growing prefix of the stream (the header is
    usually one or two BGZF blocks) -> (header dict, prefix bytes)."""
    n = min(ss.length, 1 << 20)
    while True:
        head = ss.read_at(0, n)
        h = ctx.parse_header(head)
        if isinstance(h, dict) or n >= ss.length:
            return h, head
        n = min(ss.length, 4 * n)


# ---- split guessers ------------------------------------------------------------------
class BAMSplitGuesser:
    """BAMSplitGuesser.java:50-398 (one device wave per guess).  A guess reads only its window
    (hbam_guess_window_len bytes at beg, :114-125) from the stream and hands it to
    hbam_guess_windows."""

    def __init__(self, ss, conf=None, header_stream=None):
        self.ss = SeekableFile(ss)
        self.conf = conf or Configuration()
        self.ctx = context(conf)
        h, _ = read_header_prefix(self.ss if header_stream is None else SeekableFile(header_stream), self.ctx)
        if isinstance(h, int):
            raise_for(h, "cannot read SAM header")
        self.n_ref = h["n_ref"]
        if header_stream is None and self.ss.read_at(0, 4) != b"\x1f\x8b\x08\x04":
            raise SAMFormatException("Does not seem like a BAM file")

    def guessNextBAMRecordStart(self, beg, end):
        wl = self.ctx.guess_window_len(self.ss.length, beg, end)
        w = self.ss.read_at(beg, wl)
        rc, out, err = self.ctx.guess_windows(w, [0, wl], self.ss.length, [beg], [end], self.n_ref)
        raise_for(rc, self.ctx.last_error())
        raise_for(int(err[0]), "exception escaped the guesser")
        return int(out[0])


class BGZFSplitGuesser:
    """util/BGZFSplitGuesser.java:30-148; a guess reads its one window (:62-63)."""

    def __init__(self, inp, conf=None):
        self.ss = SeekableFile(inp)
        self.ctx = context(conf)

    def guessNextBGZFBlockStart(self, beg, end):
        wl = self.ctx.guess_bgzf_window_len(self.ss.length, beg, end)
        r, e = self.ctx.guess_bgzf_window(self.ss.read_at(beg, wl), self.ss.length, beg, end)
        raise_for(e, "exception escaped the guesser")
        return int(r)


class SplittingBAMIndexer:
    """SplittingBAMIndexer.java:146-248 on the device: index(bam_bytes, out) writes the
    big-endian u64 entries (first record voffset, every granularity-th record's voffset,
    file_len<<16) that SplittingBAMIndex reads."""

    DEFAULT_GRANULARITY = 4096

    def __init__(self, granularity=DEFAULT_GRANULARITY, ctx=None):
        self.granularity = int(granularity)
        self.ctx = ctx

    def index(self, data, out=None):
        from ._lib import Context
        ctx = self.ctx or Context(0)
        rc, offs = ctx.splitting_index(data, self.granularity)
        raise_for(rc, ctx.last_error())
        raw = b"".join(struct.pack(">q", int(x)) for x in offs)
        if out is not None:
            out.write(raw)
        return raw


class SplittingBAMIndex:
    """SplittingBAMIndex.java:50-77 — big-endian u64 voffsets + file_len<<16."""

    def __init__(self, inp=None):
        self.offsets = []
        if inp is not None:
            self.readIndex(inp)

    def readIndex(self, inp):
        data = inp.read() if hasattr(inp, "read") else _read_file(inp)
        prev = -1
        self.offsets = []
        for i in range(0, len(data) - 7, 8):
            cur = struct.unpack(">q", data[i:i + 8])[0]
            if prev > cur:
                raise IOException("Invalid splitting BAM index; offsets not in order")
            self.offsets.append(cur)
            prev = cur
        if len(self.offsets) < 2:
            raise IOException("Invalid splitting BAM index: should contain at least 1 offset "
                              "and the file size")

    def prevAlignment(self, file_pos):
        import bisect
        k = bisect.bisect_right(self.offsets, file_pos << 16)
        return self.offsets[k - 1] if k else None

    def nextAlignment(self, file_pos):
        import bisect
        k = bisect.bisect_right(self.offsets, file_pos << 16)
        return self.offsets[k] if k < len(self.offsets) else None

    def size(self):
        return len(self.offsets)


class BGZFBlockIndexer:
    """util/BGZFBlockIndexer.java:41-225 on the device: index(bgzf_bytes, out) writes, for
    every granularity-th block, the offset after it as a big-endian 48-bit integer, then the
    file length ([file].bgzfi).  Like the reference, offsets past 2 GiB wrap (int `pos`)."""

    def __init__(self, granularity, ctx=None):
        if int(granularity) <= 0:
            raise IllegalArgumentException(
                "Granularity must be a positive integer, not '%s'!" % granularity)
        self.granularity = int(granularity)
        self.ctx = ctx

    def index(self, data, out=None):
        ctx = self.ctx or context()
        if isinstance(data, str):
            path, data = data, _read_file(data)
        else:
            path = None
        rc, offs = ctx.bgzf_block_index(data, self.granularity)
        raise_for(rc, ctx.last_error())
        raw = b"".join(struct.pack(">q", int(x))[2:] for x in offs)
        if out is None and path is not None:
            with open(path + ".bgzfi", "wb") as f:
                f.write(raw)
        elif out is not None:
            out.write(raw)
        return raw


class BGZFBlockIndex:
    """util/BGZFBlockIndex.java:39-78 — 48-bit big-endian block offsets + the file size."""

    def __init__(self, inp=None):
        self.offsets = []
        if inp is not None:
            self.readIndex(inp)

    def readIndex(self, inp):  # :50-69
        data = inp.read() if hasattr(inp, "read") else _read_file(inp)
        prev = -1
        offs = set()
        for i in range(0, len(data) - 5, 6):
            cur = int.from_bytes(data[i:i + 6], "big")
            if prev > cur:
                raise IOException("Invalid BGZF block index; offsets not in order: %#x > %#x"
                                  % (prev, cur))
            offs.add(cur)
            prev = cur
        if len(offs) < 1:
            raise IOException("Invalid BGZF block index: should contain at least the file size")
        offs.add(0)
        self.offsets = sorted(offs)

    def prevBlock(self, file_pos):  # TreeSet.floor
        import bisect
        k = bisect.bisect_right(self.offsets, file_pos)
        return self.offsets[k - 1] if k else None

    def nextBlock(self, file_pos):  # TreeSet.higher
        import bisect
        k = bisect.bisect_right(self.offsets, file_pos)
        return self.offsets[k] if k < len(self.offsets) else None

    def size(self):
        return len(self.offsets)

    def fileSize(self):
        return self.offsets[-1]


class BGZFSplitFileInputFormat:
    """util/BGZFSplitFileInputFormat.java:50-170: Hadoop FileSplits aligned to BGZF block
    starts, from [path].bgzfi when present, else by BGZFSplitGuesser (device)."""

    @staticmethod
    def getIdxPath(path):
        return str(path) + ".bgzfi"

    def getSplits(self, splits, cfg=None):  # :51-81
        cfg = cfg or Configuration()
        splits = sorted(splits, key=lambda s: str(s.getPath()))
        out, i = [], 0
        while i < len(splits):
            try:
                i = self._add_indexed_splits(splits, i, out, cfg)
            except IOException:
                i = self._add_probabilistic_splits(splits, i, out, cfg)
        return out

    def _add_indexed_splits(self, splits, i, out, cfg):  # :85-122
        path = splits[i].getPath()
        try:
            with open(self.getIdxPath(path), "rb") as f:
                idx = BGZFBlockIndex(f)
        except OSError as e:
            raise IOException(str(e))
        j_end = i
        while j_end < len(splits) and splits[j_end].getPath() == path:
            j_end += 1
        for j in range(i, j_end):
            fs = splits[j]
            start, end = fs.getStart(), fs.getStart() + fs.getLength()
            bs = idx.prevBlock(start)
            be = idx.prevBlock(end) if j == j_end - 1 else idx.nextBlock(end)
            if bs is None:
                raise JavaRuntimeException("Internal error or invalid index: no block start for %d" % start)
            if be is None:
                raise JavaRuntimeException("Internal error or invalid index: no block end for %d" % end)
            out.append(FileSplit(path, bs, be - bs, fs.getLocations()))
        return j_end

    def _add_probabilistic_splits(self, splits, i, out, cfg):  # :126-153
        path = splits[i].getPath()
        guesser = BGZFSplitGuesser(path, cfg)
        while True:  # do { ... } while (i < size && fspl.getPath().equals(path))
            fs = splits[i]
            beg, end = fs.getStart(), fs.getStart() + fs.getLength()
            aligned = guesser.guessNextBGZFBlockStart(beg, end)
            out.append(FileSplit(path, aligned, end - aligned, fs.getLocations()))
            i += 1
            if not (i < len(splits) and fs.getPath() == path):
                break
        return i

    def isSplitable(self, job=None, path=None):
        return True


# ---- record value -------------------------------------------------------------------
class SAMRecordWritable:
    """SAMRecordWritable.java:46-70."""

    def __init__(self):
        self.record = None

    def get(self):
        return self.record

    def set(self, r):
        self.record = r

    def write(self, out):
        out.write(self.record.toBAMBytes())

    def readFields(self, inp):  # :66-69, lazy decode (LazyBAMRecordFactory)
        bs = struct.unpack("<i", inp.read(4))[0]
        body = inp.read(bs)
        self.record = BAMRecordBytes(struct.pack("<i", bs) + body)


class BAMRecordBytes:
    """A lazily decoded BAM record over its wire bytes (block_size + record), as
    SAMRecordWritable.readFields builds it with LazyBAMRecordFactory (LazyBAMRecordFactory.java
    :31-99): fixed fields are read on access, the variable block is kept verbatim."""

    def __init__(self, raw):
        self.raw = bytes(raw)
        (self._bs, self._ref, self._pos, self._lrn, self._mapq, self._bin, self._ncig, self._flag,
         self._lseq, self._nref, self._npos, self._tlen) = struct.unpack_from("<iiiBBHHHiiii", self.raw, 0)

    def toBAMBytes(self):
        return self.raw

    def getVariableBinaryRepresentation(self):
        return self.raw[36:]

    def getReferenceIndex(self):
        return self._ref

    def getAlignmentStart(self):
        return _i32(self._pos + 1)

    def getFlags(self):
        return self._flag

    def getReadUnmappedFlag(self):
        return bool(self._flag & 4)

    def getMappingQuality(self):
        return self._mapq

    def getMateReferenceIndex(self):
        return self._nref

    def getMateAlignmentStart(self):
        return _i32(self._npos + 1)

    def getInferredInsertSize(self):
        return self._tlen

    def getIndexingBin(self):
        return self._bin

    def _var(self):
        v = self.raw[36:]
        p = self._lrn
        cig = v[p:p + 4 * self._ncig]
        p += 4 * self._ncig
        seq = v[p:p + (self._lseq + 1) // 2]
        p += (self._lseq + 1) // 2
        return v, cig, seq, v[p:p + self._lseq]

    def getReadName(self):
        return self.raw[36:36 + max(self._lrn - 1, 0)].decode("latin-1")

    def getCigarString(self):
        _, cig, _, _ = self._var()
        ops = struct.unpack("<%dI" % (len(cig) // 4), cig)
        return "".join("%d%s" % (o >> 4, "MIDNSHP=X"[o & 15]) for o in ops) or "*"

    def getReadString(self):
        _, _, seq, _ = self._var()
        a = "=ACMGRSVTWYHKDBN"
        out = "".join(a[b >> 4] + a[b & 15] for b in seq)[:self._lseq]
        return out or "*"

    def getReadBases(self):
        s = self.getReadString()
        return s.encode() if s != "*" else b""

    def getBaseQualities(self):
        return self._var()[3]


class LongWritable:
    def __init__(self, v=0):
        self.v = int(v)

    def get(self):
        return self.v

    def set(self, v):
        self.v = int(v)


# ---- the record reader ---------------------------------------------------------------
_M64 = (1 << 64) - 1
_C1, _C2 = 0x87c37b91114253d5, 0x4cf5ad432745937f


def _rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & _M64


def _fmix(k):
    k ^= k >> 33
    k = (k * 0xff51afd7ed558ccd) & _M64
    k ^= k >> 33
    k = (k * 0xc4ceb9fe1a85ec53) & _M64
    return k ^ (k >> 33)


def _s64(x):
    return x - (1 << 64) if x >> 63 else x


def _finish(h1, h2, n):
    h1 ^= n & _M64
    h2 ^= n & _M64
    h1 = (h1 + h2) & _M64
    h2 = (h2 + h1) & _M64
    h1, h2 = _fmix(h1), _fmix(h2)
    return _s64((h1 + h2) & _M64)


def _mix_block(h1, h2, k1, k2):
    k1 = (k1 * _C1) & _M64
    k1 = (_rotl(k1, 31) * _C2) & _M64
    h1 ^= k1
    h1 = (_rotl(h1, 27) + h2) & _M64
    h1 = (h1 * 5 + 0x52dce729) & _M64
    k2 = (k2 * _C2) & _M64
    k2 = (_rotl(k2, 33) * _C1) & _M64
    h2 ^= k2
    h2 = ((h2 << 31) | (h1 >> 33)) & _M64  # MurmurHash3.java:59 mixes h1 in here
    h2 = (h2 + h1) & _M64
    h2 = (h2 * 5 + 0x38495ab5) & _M64
    return h1, h2


def murmurhash3_bytes(key, seed=0):
    """util/MurmurHash3.java:32-102 (byte[] variant, incl. the line-59 h2 quirk)."""
    key = bytes(key)
    n = len(key)
    h1 = h2 = seed & _M64
    nb = n // 16
    for i in range(nb):
        k1, k2 = struct.unpack_from("<QQ", key, 16 * i)
        h1, h2 = _mix_block(h1, h2, k1, k2)
    t = key[16 * nb:]
    k1 = k2 = 0
    if len(t) > 8:
        for j in range(len(t) - 1, 7, -1):
            k2 ^= t[j] << (8 * (j - 8))
        k2 = (_rotl((k2 * _C2) & _M64, 33) * _C1) & _M64
        h2 ^= k2
    if len(t):
        for j in range(min(len(t), 8) - 1, -1, -1):
            k1 ^= t[j] << (8 * j)
        k1 = (_rotl((k1 * _C1) & _M64, 31) * _C2) & _M64
        h1 ^= k1
    return _finish(h1, h2, n)


def murmurhash3_chars(chars, seed=0):
    """util/MurmurHash3.java:108-171 (CharSequence variant: UTF-16 code units; the tail reads
    charAt(0..6) from the START of the sequence, as the reference does)."""
    c = [ord(x) for x in str(chars)]
    n = len(c)
    h1 = h2 = seed & _M64
    for i in range(n // 8):
        i0, i1 = 8 * i, 8 * i + 4
        k1 = c[i0] | c[i0 + 1] << 16 | c[i0 + 2] << 32 | c[i0 + 3] << 48
        k2 = c[i1] | c[i1 + 1] << 16 | c[i1 + 2] << 32 | c[i1 + 3] << 48
        h1, h2 = _mix_block(h1, h2, k1, k2)
    r = n & 7
    k1 = k2 = 0
    if r >= 5:
        for j in range(r - 1, 3, -1):
            k2 ^= c[j] << (16 * (j - 4))
        k2 = (_rotl((k2 * _C2) & _M64, 33) * _C1) & _M64
        h2 ^= k2
    if r >= 1:
        for j in range(min(r, 4) - 1, -1, -1):
            k1 ^= c[j] << (16 * j)
        k1 = (_rotl((k1 * _C1) & _M64, 31) * _C2) & _M64
        h1 ^= k1
    return _finish(h1, h2, n)


def _i32(x):
    x &= 0xffffffff
    return x - (1 << 32) if x >> 31 else x


class _DecodedSplit:
    """One window's host copy (hbam_records_to_host: key, voffset, rec_off, block_size and the
    records' bytes — views of the context's pinned staging, valid until the next window)."""

    def __init__(self, cols):
        self.cols = cols
        self.ubuf = cols.get("ubuf")

    def record_bytes(self, i):
        r = int(self.cols["rec_off"][i])
        return bytes(self.ubuf[r:r + 4 + int(self.cols["block_size"][i])])

    def var_block(self, i):
        r = int(self.cols["rec_off"][i])
        return bytes(self.ubuf[r + 36:r + 4 + int(self.cols["block_size"][i])])


WINDOW_BYTES_PROPERTY = "hadoopbam.hip.window-bytes"


def read_header(data, ctx):
    """SAMHeaderReader.readSAMHeaderFrom (util/SAMHeaderReader.java:53-72) on the device, from a
    growing prefix of the file (the header is usually one or two BGZF blocks)."""
    n = min(len(data), 1 << 20)
    while True:
        h = ctx.parse_header(data[:n])
        if isinstance(h, dict) or n >= len(data):
            return h
        n = min(len(data), 4 * n)


class BAMRecordReader:
    """BAMRecordReader.java:48-188.  initialize() opens a streamed device decode of the split
    (hbam_split_open: windows of hadoopbam.hip.window-bytes compressed bytes, the next one
    copied while the current one decodes); each window's records come to the host through
    hbam_records_to_host (key, voffset, record bytes only); nextKeyValue() walks them and
    raises the reference's exception at the record where the reference raises it.  The key
    and value objects are reused, as in the reference (:53-54, :185-186)."""

    def __init__(self):
        self.key = LongWritable()
        self.record = SAMRecordWritable()
        self._init = False
        self._gen = None

    @staticmethod
    def getKey0(ref_idx, alignment_start0):
        """(long)refIdx << 32 | alignmentStart0 — the int is sign-extended (:104-106)."""
        v = (int(np.int32(ref_idx)) << 32) | int(np.int32(alignment_start0))
        return ((v + (1 << 63)) % (1 << 64)) - (1 << 63)

    @staticmethod
    def getKey(rec, alignment_start=None):
        """getKey(SAMRecord) (:66-96) or getKey(int refIdx, int alignmentStart) (:99-101)."""
        if alignment_start is not None:
            return BAMRecordReader.getKey0(rec, _i32(int(alignment_start) - 1))
        ref_idx = int(rec.getReferenceIndex())
        start = int(rec.getAlignmentStart())
        if not (rec.getReadUnmappedFlag() or ref_idx < 0 or start < 0):
            return BAMRecordReader.getKey0(ref_idx, _i32(start - 1))
        var = rec.getVariableBinaryRepresentation()
        if var is not None:  # undecoded BAM record: hash its raw variable block
            h = _i32(murmurhash3_bytes(var, 0))
        else:  # decoded record: a few representative fields, chained (:88-93)
            h = _i32(murmurhash3_chars(rec.getReadName(), 0))
            h = _i32(murmurhash3_bytes(rec.getReadBases(), h))
            h = _i32(murmurhash3_bytes(rec.getBaseQualities(), h))
            h = _i32(murmurhash3_chars(rec.getCigarString(), h))
        return BAMRecordReader.getKey0(0x7fffffff, h)

    def initialize(self, split, ctx=None):
        if self._init:
            self.close()
        self._init = True
        conf = ctx if isinstance(ctx, Configuration) else Configuration()
        self.split = split
        path = split.getPath()
        data = path if isinstance(path, (bytes, bytearray, np.ndarray)) else np.memmap(path, np.uint8, "r")
        self._data = data
        self.ctxt = context(conf)
        h = read_header(data, self.ctxt)
        if isinstance(h, int):
            raise_for(h, "cannot read SAM header")
        window = int(conf.get(WINDOW_BYTES_PROPERTY, 1 << 30))
        if isinstance(data, np.memmap):
            # a file: split-local positioned reads (the reference seeks an FSDataInputStream,
            # :128-143, WrapSeekable.java:42-87) — only the blocks the split needs are read
            self._fd = os.open(path, os.O_RDONLY)
            fd = self._fd
            self._gen = self.ctxt.split_stream_reader(lambda off, n: os.pread(fd, n, off), len(data),
                                                      split.getStartVirtualOffset(),
                                                      split.getEndVirtualOffset(), h["n_ref"], window,
                                                      host="records")
        else:
            self._gen = self.ctxt.split_stream(data, split.getStartVirtualOffset(),
                                               split.getEndVirtualOffset(), h["n_ref"], window,
                                               host="records")
        self.dec = None
        self.i = self.n = 0
        self.status = 0
        self._last = False
        self.file_start = split.getStartVirtualOffset() >> 16
        self.v_end = split.getEndVirtualOffset()
        self._next_window()

    def _next_window(self):
        try:
            cols = next(self._gen)
        except StopIteration:
            self._last = True
            self.dec, self.i, self.n, self.status = None, 0, 0, 0
            return False
        self.dec = _DecodedSplit(cols)
        self.i, self.n, self.status = 0, cols["n"], cols["status"]
        if self.status != 0:
            self._last = True
        return True

    def nextKeyValue(self):
        while self.dec is not None and self.i >= self.n:
            if self.status != 0:
                st, self.status = self.status, 0
                raise_for(st, "at record %d of the window" % self.n)
            if self._last or not self._next_window():
                return False
        if self.dec is None:
            return False
        i = self.i
        self.i += 1
        self.key.set(int(self.dec.cols["key"][i]))
        # the value is the lazily decoded record over the record's bytes, as the reference's codec
        # builds it (:172-188)
        self.record.set(BAMRecordBytes(self.dec.record_bytes(i)))
        return True

    def getCurrentKey(self):
        return self.key

    def getCurrentValue(self):
        return self.record

    def getProgress(self):  # :157-168
        if self.dec is None or self.i >= self.n:
            return 1.0 if self._last else 0.0
        vp = int(self.dec.cols["voffset"][self.i])
        file_end = self.v_end >> 16
        return float((vp >> 16) - self.file_start) / (file_end - self.file_start + 1)

    def close(self):
        if self._gen is not None:
            self._gen.close()
        self._gen = None
        self.dec = None
        if getattr(self, "_fd", None) is not None:
            os.close(self._fd)
            self._fd = None


# ---- input formats -------------------------------------------------------------------
class BAMInputFormat:
    """BAMInputFormat.java:50-229."""

    def createRecordReader(self, split, ctx=None):
        rr = BAMRecordReader()
        rr.initialize(split, ctx)
        return rr

    def getSplits(self, splits, cfg=None):
        cfg = cfg or Configuration()
        splits = sorted(splits, key=lambda s: str(s.getPath()))
        out, i = [], 0
        while i < len(splits):
            try:
                i = self._add_indexed_splits(splits, i, out, cfg)
            except IOException:
                i = self._add_probabilistic_splits(splits, i, out, cfg)
        return out

    def _add_indexed_splits(self, splits, i, out, cfg):  # :107-159
        path = splits[i].getPath()
        idx_path = str(path) + ".splitting-bai"
        if not os.path.exists(idx_path):
            raise IOException("no index")
        with open(idx_path, "rb") as f:
            idx = SplittingBAMIndex(f)
        j_end = i
        while j_end < len(splits) and splits[j_end].getPath() == path:
            j_end += 1
        pot = []
        for j in range(i, j_end):
            fs = splits[j]
            start, end = fs.getStart(), fs.getStart() + fs.getLength()
            bs = idx.nextAlignment(start)
            be = (idx.prevAlignment(end) | 0xffff) if j == j_end - 1 else idx.nextAlignment(end)
            if bs is None or be is None:
                return self._add_probabilistic_splits(splits, i, out, cfg)
            pot.append(FileVirtualSplit(path, bs, be, fs.getLocations()))
        out.extend(pot)
        return j_end

    def _add_probabilistic_splits(self, splits, i, out, cfg):  # :163-224
        """The guesses of one file's FileSplits as one hbam_probabilistic_splits_windows call:
        the header prefix and each split's guess window are read from the file, nothing else."""
        path = splits[i].getPath()
        ss = SeekableFile(path)
        ctx = context(cfg)
        j = i
        beg, end = [], []
        while j < len(splits) and splits[j].getPath() == path:
            beg.append(splits[j].getStart())
            end.append(splits[j].getStart() + splits[j].getLength())
            j += 1
        lens = [ctx.guess_window_len(ss.length, b, e) for b, e in zip(beg, end)]
        win_off = np.zeros(len(lens) + 1, np.uint64)
        win_off[1:] = np.cumsum(lens)
        windows = b"".join(ss.read_at(b, n) for b, n in zip(beg, lens))
        hn = min(ss.length, 1 << 20)
        while True:
            n, vs, ve = ctx.probabilistic_splits_windows(ss.read_at(0, hn), windows, win_off,
                                                         ss.length, beg, end)
            if n != _lib.HBAM_ETRUNC or hn >= ss.length:
                break
            hn = min(ss.length, 4 * hn)
        ss.close()
        if n < 0:
            raise_for(int(n), ctx.last_error())
        # each virtual split carries the locations of the FileSplit whose guess opened it
        # (:201-203): the guess for split j lands in [beg_j, end_j), so the owner is the last j
        # with beg_j <= the start's compressed offset
        owners = np.searchsorted(np.asarray(beg, np.int64),
                                 (np.asarray(vs, np.uint64) >> np.uint64(16)).astype(np.int64),
                                 side="right") - 1
        for a, b, o in zip(vs, ve, owners):
            out.append(FileVirtualSplit(path, int(a), int(b), splits[i + max(int(o), 0)].getLocations()))
        return j

    def isSplitable(self, job=None, path=None):
        return True


class AnySAMInputFormat(BAMInputFormat):
    """AnySAMInputFormat.java:52-243 — BAM by extension or the 0x1f first byte."""

    TRUST_EXTS_PROPERTY = "hadoopbam.anysam.trust-exts"

    def getFormat(self, path, conf=None):
        conf = conf or Configuration()
        trust = str(conf.get(self.TRUST_EXTS_PROPERTY, "true")).lower() != "false"
        if trust and str(path).endswith(".bam"):
            return "BAM"
        with open(path, "rb") as f:
            b = f.read(1)
        if b == b"\x1f":
            return "BAM"
        if b == b"@":
            return "SAM"
        return None
