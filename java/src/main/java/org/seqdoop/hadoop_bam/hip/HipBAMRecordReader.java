// Drop-in body of org.seqdoop.hadoop_bam.BAMRecordReader (BAMRecordReader.java:48-188) over
// the C ABI.  initialize() reads the header as the reference does (:128-130) and opens a
// streamed device decode of the FileVirtualSplit (hbam_split_open_reader: windows of
// hadoopbam.hip.window-bytes compressed bytes, the next copied while the current decodes, each
// read from the FSDataInputStream by positioned reads of the split's own bytes, SplitSource);
// nextKeyValue() hands out (LongWritable key, SAMRecordWritable) from each window's host
// columns and throws the reference's exception at the record where the reference would.
// The value is the lazily decoded BAMRecord htsjdk would build from the same record bytes.
package org.seqdoop.hadoop_bam.hip;

import java.io.ByteArrayInputStream;
import java.io.IOException;
import java.lang.foreign.*;

import org.apache.hadoop.conf.Configuration;
import org.apache.hadoop.fs.FSDataInputStream;
import org.apache.hadoop.fs.FileSystem;
import org.apache.hadoop.fs.Path;
import org.apache.hadoop.io.LongWritable;
import org.apache.hadoop.mapreduce.InputSplit;
import org.apache.hadoop.mapreduce.RecordReader;
import org.apache.hadoop.mapreduce.TaskAttemptContext;

import htsjdk.samtools.BAMRecordCodec;
import htsjdk.samtools.SAMFileHeader;
import htsjdk.samtools.SAMRecord;
import htsjdk.samtools.ValidationStringency;
import htsjdk.samtools.util.RuntimeIOException;

import hbparquet.hadoop.util.ContextUtil;
import org.seqdoop.hadoop_bam.FileVirtualSplit;
import org.seqdoop.hadoop_bam.SAMRecordWritable;
import org.seqdoop.hadoop_bam.util.SAMHeaderReader;

public class HipBAMRecordReader extends RecordReader<LongWritable, SAMRecordWritable> {
  public static final String WINDOW_BYTES_PROPERTY = "hadoopbam.hip.window-bytes";
  public static final String DEVICE_PROPERTY = "hadoopbam.hip.device";

  private static final ThreadLocal<Hbam> SPLIT_CTX = new ThreadLocal<Hbam>();

  /** The split side's context: one per client thread (the guessers, like the reference's, are
   *  not thread-safe), CRC checks on as in both guessers (BAMSplitGuesser.java:130). */
  static Hbam context(Configuration conf) throws IOException {
    Hbam h = SPLIT_CTX.get();
    if (h == null) {
      h = new Hbam(conf.getInt(DEVICE_PROPERTY, 0), true);
      SPLIT_CTX.set(h);
    }
    return h;
  }

  private final LongWritable key = new LongWritable();
  private final SAMRecordWritable record = new SAMRecordWritable();
  private boolean isInitialized = false;

  private Hbam hbam;
  private Arena arena;               // file mapping + column structs of this reader
  private MemorySegment stream;      // hbam_split_stream*
  private MemorySegment dev, host;   // hbam_columns: device (library-owned) / host copy
  private boolean hostLive = false, last = false;
  private long n, i;
  private int status;
  private MemorySegment keys, recOff, blockSize, ubuf, voffs;
  private BAMRecordCodec codec;
  private ValidationStringency stringency;
  private long fileStart, virtualEnd;
  private int[] mergeMap;            // HipSortRecordReader: merged index of each input index, or null
  private SplitSource source;        // positioned reads of the split's bytes (hbam_read_fn upcalls)

  /** Utils.correctSAMRecordForMerging on the device for every window (hbam_merge_remap):
   *  SortRecordReader (Sort.java:279-295) sets it when the inputs' dictionaries differ. */
  void setMergeMap(int[] map) { mergeMap = map; }

  /** Utils.correctSAMRecordForMerging's PG / RG rewrite on the device (hbam_rewrite_groups) with
   *  the table HipSortRecordReader builds from htsjdk's own merger. */
  void setGroupTable(byte[] table) { groupTable = table; }
  private byte[] groupTable;
  private int groupStatus = Hbam.OK;

  SAMFileHeader header() { return codecHeader; }
  private SAMFileHeader codecHeader;

  @Override public void initialize(InputSplit spl, TaskAttemptContext ctx) throws IOException {
    if (isInitialized) close();  // re-entrant, as the reference (:116-118)
    isInitialized = true;
    final Configuration conf = ContextUtil.getConfiguration(ctx);
    final FileVirtualSplit split = (FileVirtualSplit) spl;
    final Path file = split.getPath();
    final FileSystem fs = file.getFileSystem(conf);
    this.stringency = SAMHeaderReader.getValidationStringency(conf);

    final SAMFileHeader header;
    try (FSDataInputStream in = fs.open(file)) {
      header = SAMHeaderReader.readSAMHeaderFrom(in, conf);
    }
    // the lazy record of each hand-out is built from the record's bytes by htsjdk's own codec
    codec = new BAMRecordCodec(header);
    codecHeader = header;
    final int nRef = header.getSequenceDictionary().size();
    final long len = fs.getFileStatus(file).getLen();

    arena = Arena.ofShared();
    hbam = new Hbam(conf.getInt(DEVICE_PROPERTY, 0), false);
    fileStart = split.getStartVirtualOffset() >>> 16;
    virtualEnd = split.getEndVirtualOffset();
    // only the split's blocks are read (into the library's pinned staging, so each window's copy
    // overlaps the previous window's decode), as the reference's seek + read (:128-143)
    source = new SplitSource(fs, file, arena);
    stream = source.open(hbam, len, split.getStartVirtualOffset(), virtualEnd, nRef,
                         conf.getLong(WINDOW_BYTES_PROPERTY, 1L << 30));
    dev = arena.allocate(Hbam.COLUMNS);
    host = arena.allocate(Hbam.COLUMNS);
    n = i = 0;
    status = Hbam.OK;
    last = false;
    nextWindow();
  }

  private static MemorySegment ptr(MemorySegment cols, String f, long bytes) {
    return cols.get(ValueLayout.ADDRESS, Hbam.offsetOf(f)).reinterpret(Math.max(bytes, 1));
  }

  /** The next window's records (hbam_split_next + hbam_split_records_to_host); false at the end. */
  private boolean nextWindow() {
    long bad = -1;  // first record hbam_merge_remap refuses (HipSortRecordReader only)
    try {
      hostLive = false;  // the previous window's host copy is the stream's staging: reused below
      final int rc = (int) Hbam.SPLIT_NEXT.invokeExact(stream, dev);
      if (rc < 0) {
        if (source.failure() != null) throw new RuntimeIOException(source.failure());
        throw new RuntimeIOException("hbam_split_next: " + hbam.lastError());
      }
      if (rc == 0) { last = true; n = i = 0; return false; }
      if (mergeMap != null) {
        try (Arena a = Arena.ofConfined()) {
          final MemorySegment m = a.allocateFrom(ValueLayout.JAVA_INT, mergeMap);
          final MemorySegment b = a.allocate(ValueLayout.JAVA_LONG);
          final int rc3 = (int) Hbam.MERGE_REMAP.invokeExact(hbam.context(), dev, m, mergeMap.length, b);
          if (rc3 != Hbam.OK) throw new RuntimeIOException("hbam_merge_remap: " + hbam.lastError());
          bad = b.get(ValueLayout.JAVA_LONG, 0);
        }
      }
      if (groupTable != null) {
        // correctSAMRecordForMerging runs per record (cli/Utils.java:286-324): the records before
        // the one setReferenceIndex refuses still get their group rewrite, so the rewrite covers
        // [0, bad) and an exception it raises at an earlier record is the one thrown
        if (bad >= 0 && bad < dev.get(ValueLayout.JAVA_LONG, Hbam.offsetOf("n_records")))
          dev.set(ValueLayout.JAVA_LONG, Hbam.offsetOf("n_records"), bad);
        try (Arena a = Arena.ofConfined()) {
          final MemorySegment t = a.allocateFrom(ValueLayout.JAVA_BYTE, groupTable);
          final MemorySegment st = a.allocate(ValueLayout.JAVA_INT), er = a.allocate(ValueLayout.JAVA_LONG);
          final int rc4 = (int) Hbam.REWRITE_GROUPS.invokeExact(hbam.context(), dev, t, (long) groupTable.length, st, er);
          if (rc4 != Hbam.OK) throw new RuntimeIOException("hbam_rewrite_groups: " + hbam.lastError());
          groupStatus = st.get(ValueLayout.JAVA_INT, 0);
        }
      }
      // only what nextKeyValue reads: key, voffset, rec_off, block_size and the record bytes, into
      // the split stream's pinned staging (hbam_split_records_to_host; no pool crosses PCIe)
      final int rc2 = (int) Hbam.SPLIT_RECORDS_TO_HOST.invokeExact(stream, dev, host);
      if (rc2 != Hbam.OK) throw new RuntimeIOException("hbam_split_records_to_host: " + hbam.lastError());
      hostLive = true;
    } catch (RuntimeException e) {
      throw e;
    } catch (Throwable t) {
      throw new RuntimeIOException(t);
    }
    n = host.get(ValueLayout.JAVA_LONG, Hbam.offsetOf("n_records"));
    status = host.get(ValueLayout.JAVA_INT, Hbam.offsetOf("status"));
    final int gs = groupStatus;
    groupStatus = Hbam.OK;
    if (gs != Hbam.OK) {
      // the rewrite stopped at record n (dv holds the records before it), before any `bad`
      status = gs;
    } else if (mergeMap != null && bad >= 0 && bad <= n) {
      // SAMRecord.setReferenceIndex against the record's own header throws here (:286-313)
      n = bad;
      status = Hbam.EREFID;
    }
    if (status != Hbam.OK) last = true;
    i = 0;
    keys = ptr(host, "key", 8 * n);
    voffs = ptr(host, "voffset", 8 * n);
    recOff = ptr(host, "rec_off", 8 * n);
    blockSize = ptr(host, "block_size", 4 * n);
    ubuf = ptr(host, "ubuf", host.get(ValueLayout.JAVA_LONG, Hbam.offsetOf("ubuf_len")));
    return true;
  }

  @Override public boolean nextKeyValue() {
    while (i >= n) {
      if (status != Hbam.OK) {  // raised at the record where the reference raises it
        final int s = status;
        status = Hbam.OK;
        throw Hbam.exceptionFor(s, "BAMRecordReader.nextKeyValue");
      }
      if (last || !nextWindow()) return false;
    }
    final long off = recOff.getAtIndex(ValueLayout.JAVA_LONG, i);
    final int bs = blockSize.getAtIndex(ValueLayout.JAVA_INT, i);
    final byte[] raw = ubuf.asSlice(off, 4L + bs).toArray(ValueLayout.JAVA_BYTE);
    codec.setInputStream(new ByteArrayInputStream(raw));
    final SAMRecord r = codec.decode();  // exactly the bytes the reference's codec reads
    if (stringency != null) r.setValidationStringency(stringency);
    key.set(keys.getAtIndex(ValueLayout.JAVA_LONG, i));  // = BAMRecordReader.getKey(r)
    record.set(r);
    ++i;
    return true;
  }

  @Override public LongWritable getCurrentKey() { return key; }
  @Override public SAMRecordWritable getCurrentValue() { return record; }

  @Override public float getProgress() {  // :157-168, from the next record's voffset
    if (i >= n) return last ? 1 : 0;
    final long filePos = voffs.getAtIndex(ValueLayout.JAVA_LONG, i) >>> 16;
    final long fileEnd = virtualEnd >>> 16;
    return (float) (filePos - fileStart) / (fileEnd - fileStart + 1);
  }

  @Override public void close() throws IOException {
    try {
      if (stream != null && stream.address() != 0) Hbam.SPLIT_CLOSE.invokeExact(stream);
      if (source != null) source.close();
    } catch (Throwable t) {
      throw new IOException(t);
    } finally {
      hostLive = false;
      stream = null;
      source = null;
      if (hbam != null) hbam.close();
      hbam = null;
      if (arena != null) arena.close();
      arena = null;
    }
  }
}
