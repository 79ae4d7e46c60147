"""BAM output with the device BGZF compressor (hbam_bgzf_compress):
mirrors BAMRecordWriter (BAMRecordWriter.java:48-141), KeyIgnoringBAMRecordWriter,
KeyIgnoringBAMOutputFormat (KeyIgnoringBAMOutputFormat.java:43-98),
util.SAMOutputPreparer.prepareForRecords (:58-95) and cli.Utils.mergeSAMInto (:333-356)
— the pieces the Sort plugin uses to write its sorted BAM.

The compressed bytes are the device compressor's, not zlib's: what the reference's tests
check, and what these classes guarantee, is the inflated stream (header bytes, then every
record's BAMRecordCodec.encode bytes in write order) and the BGZF framing (members of at most
65280 inflated bytes, the 28-byte EOF block only where the reference writes it)."""
import io
import os
import struct

import numpy as np

from . import _lib

BAM_MAGIC = b"BAM\x01"
EMPTY_GZIP_BLOCK = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
_FLUSH_BYTES = 256 << 20  # host bytes buffered before a device compression


class SAMFileHeader:
    """The parts of htsjdk's SAMFileHeader the BAM writer serializes: the text and the
    sequence dictionary (name, length)."""

    def __init__(self, text, refs):
        self.text = text if isinstance(text, bytes) else text.encode()
        self.refs = [(n if isinstance(n, bytes) else n.encode(), int(l)) for n, l in refs]

    @classmethod
    def from_bam_bytes(cls, b):
        """Parse the inflated header of a BAM (BAMFileReader.readHeader layout)."""
        if bytes(b[:4]) != BAM_MAGIC:
            raise IOError("not a BAM header")
        l_text = struct.unpack_from("<i", b, 4)[0]
        text = bytes(b[8:8 + l_text])
        p = 8 + l_text
        n_ref = struct.unpack_from("<i", b, p)[0]
        p += 4
        refs = []
        for _ in range(n_ref):
            ln = struct.unpack_from("<i", b, p)[0]
            name = bytes(b[p + 4:p + 4 + ln - 1])
            lr = struct.unpack_from("<i", b, p + 4 + ln)[0]
            refs.append((name, lr))
            p += 8 + ln
        return cls(text, refs)

    def getSequenceDictionary(self):
        return self.refs

    def setSortOrder(self, order):
        """SO: of the @HD line (Utils.setHeaderMergerSortOrder(conf, coordinate), Sort.java:111);
        an @HD line is added when absent (SAMFileHeader.setSortOrder)."""
        lines = self.text.split(b"\n")
        so = b"SO:" + order.encode()
        for i, ln in enumerate(lines):
            if ln.startswith(b"@HD"):
                f = [x for x in ln.split(b"\t") if not x.startswith(b"SO:")]
                lines[i] = b"\t".join(f + [so])
                break
        else:
            lines.insert(0, b"@HD\tVN:1.4\t" + so)
        self.text = b"\n".join(lines)

    def to_bam_bytes(self):
        """BAMRecordWriter.writeHeader (:126-141) / SAMOutputPreparer (:72-89): magic, l_text,
        text, n_ref, then per reference l_name, name NUL, l_ref (little-endian)."""
        out = [BAM_MAGIC, struct.pack("<i", len(self.text)), self.text, struct.pack("<i", len(self.refs))]
        for name, ln in self.refs:
            out += [struct.pack("<i", len(name) + 1), name, b"\x00", struct.pack("<i", ln)]
        return b"".join(out)


def read_sam_header(path_or_bytes, ctx):
    """SAMHeaderReader.readSAMHeaderFrom for a BAM: the header bytes of the inflated stream
    (device scan + inflate of the first blocks)."""
    data = path_or_bytes
    if isinstance(path_or_bytes, (str, os.PathLike)):
        with open(path_or_bytes, "rb") as f:
            data = f.read(16 << 20)
    a = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    h = ctx.parse_header(a)
    if not isinstance(h, dict):
        _lib_raise(h, ctx)
    need = int(h["header_ulen"])
    rc, blocks = ctx.scan_blocks(a)
    if rc:
        _lib_raise(rc, ctx)
    k = int(np.searchsorted(np.cumsum(blocks["isize"].astype(np.int64)), need)) + 1
    sub = {x: blocks[x][:k] for x in ("coff", "clen", "isize", "crc")}
    rc, u, off, st = ctx.inflate(a, sub, check_crc=False)
    if rc:
        _lib_raise(rc, ctx)
    return SAMFileHeader.from_bam_bytes(u[:need].tobytes())


def _lib_raise(code, ctx):
    from .formats import raise_for
    raise_for(int(code), ctx.last_error())


class _BGZFSink:
    """BlockCompressedOutputStream over an output stream: bytes are buffered on the host and
    compressed on the device in runs of whole blocks; flush() compresses the rest (a short
    block, as BlockCompressedOutputStream.flush does)."""

    def __init__(self, out, ctx, block_size=0):
        self.out, self.ctx = out, ctx
        self.bs = block_size or 65280
        self.buf = bytearray()

    def write(self, b):
        self.buf += b
        if len(self.buf) >= _FLUSH_BYTES:
            k = (len(self.buf) // self.bs) * self.bs
            self.out.write(self.ctx.bgzf_compress(bytes(self.buf[:k]), self.bs).tobytes())
            del self.buf[:k]

    def write_device(self, t, nbytes=None):
        """Record bytes already on the device (a sorted run's payload): compressed in place."""
        self.flush()
        src = t if nbytes is None else t[:nbytes]
        n = src.numel() if hasattr(src, "numel") else len(src)
        if n:
            self.out.write(self.ctx.bgzf_compress(src, self.bs).tobytes())

    def flush(self):
        if self.buf:
            self.out.write(self.ctx.bgzf_compress(bytes(self.buf), self.bs).tobytes())
            self.buf = bytearray()
        self.out.flush()


class BAMRecordWriter:
    """BAMRecordWriter.java:48-141: a BAM part written through a BGZF stream; the header is
    written when write_header, close() flushes without the EOF terminator (:113-120)."""

    def __init__(self, output, header, write_header=True, ctx=None, block_size=0):
        self._own = isinstance(output, (str, os.PathLike))
        self.orig = open(output, "wb") if self._own else output
        self.ctx = ctx or _lib.Context(0)
        self.sink = _BGZFSink(self.orig, self.ctx, block_size)
        if write_header:
            self.writeHeader(header)

    def writeHeader(self, header):
        self.sink.write(header.to_bam_bytes())

    def writeAlignment(self, rec):  # recordCodec.encode(rec) (:122-124)
        self.sink.write(rec.toBAMBytes())

    def write(self, key, value):  # KeyIgnoringBAMRecordWriter.write: the key is ignored
        self.writeAlignment(value.get())

    def write_encoded(self, raw):
        """Already-encoded records (block_size-prefixed BAM records), in order."""
        self.sink.write(bytes(raw))

    def write_device(self, t, nbytes=None):
        self.sink.write_device(t, nbytes)

    def close(self, ctx=None):
        self.sink.flush()
        if self._own:
            self.orig.close()


class KeyIgnoringBAMRecordWriter(BAMRecordWriter):
    """KeyIgnoringBAMRecordWriter.java: writes only the value of (key, SAMRecordWritable)."""


class KeyIgnoringBAMOutputFormat:
    """KeyIgnoringBAMOutputFormat.java:43-98."""

    def __init__(self):
        self.header = None
        self.writeHeader = True

    def getWriteHeader(self):
        return self.writeHeader

    def setWriteHeader(self, b):
        self.writeHeader = bool(b)

    def getSAMHeader(self):
        return self.header

    def setSAMHeader(self, header):
        self.header = header

    def readSAMHeaderFrom(self, path, ctx=None):
        self.header = read_sam_header(path, ctx or _lib.Context(0))

    def getRecordWriter(self, out, ctx=None):
        if self.header is None:
            raise IOError("Can't create a RecordWriter without the SAM header")
        return KeyIgnoringBAMRecordWriter(out, self.header, self.writeHeader, ctx)


class SAMOutputPreparer:
    """util/SAMOutputPreparer.java:58-95 for BAM: the header (magic, text, dictionary) through
    a BGZF stream, flushed; returns the stream for the records."""

    def prepareForRecords(self, out, fmt, header, ctx=None):
        if fmt != "BAM":
            raise ValueError("only BAM output is on this path")
        sink = _BGZFSink(out, ctx or _lib.Context(0))
        sink.write(header.to_bam_bytes())
        sink.flush()
        return sink


def get_mergeable_work_file(directory, base_prefix, base_postfix, work_filename, task_id, extension=""):
    """cli/Utils.getMergeableWorkFile (:176-187): prefix + work name + postfix + -%06d[.ext]."""
    return os.path.join(directory, "%s%s%s-%06d%s" % (base_prefix, work_filename, base_postfix, task_id,
                                                       "." + extension if extension else ""))


def merge_sam_into(out_path, directory, base_prefix, base_postfix, header, work_filename="",
                   ctx=None):
    """cli/Utils.mergeSAMInto (:333-356) for BAM: the merged header through its own BGZF
    stream (SAMOutputPreparer), the work files (mergeInto :194-229: glob
    prefix+work+postfix-[0-9]{6}*, in name order) copied byte for byte and deleted, then the
    BGZF EOF block.  `header` is getSAMHeaderMerger(conf).getMergedHeader() (:348-349): a
    SAMFileHeader, or the inputs' headers (a list), merged here with coordinate order (Sort)."""
    import fnmatch
    if isinstance(header, (list, tuple)):
        from .sort import SamFileHeaderMerger
        header = SamFileHeaderMerger("coordinate", header).getMergedHeader() if len(header) > 1 else header[0]
    pat = base_prefix + work_filename + base_postfix + "-" + "[0-9]" * 6 + "*"
    parts = sorted(f for f in os.listdir(directory) if fnmatch.fnmatchcase(f, pat))
    with open(out_path, "wb") as outs:
        SAMOutputPreparer().prepareForRecords(outs, "BAM", header, ctx)
        for f in parts:
            with open(os.path.join(directory, f), "rb") as fin:
                while True:
                    b = fin.read(64 << 20)
                    if not b:
                        break
                    outs.write(b)
        outs.write(EMPTY_GZIP_BLOCK)
    for f in parts:
        os.remove(os.path.join(directory, f))
