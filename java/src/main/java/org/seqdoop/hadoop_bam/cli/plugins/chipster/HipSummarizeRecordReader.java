// Drop-in body of SummarizeRecordReader (cli/plugins/chipster/Summarize.java:664-755) over the C
// ABI (SURVEY.md §8 f-4).  The base reader is the BAM read path's split stream
// (hbam_split_open_reader / hbam_split_next over SplitSource, as HipBAMRecordReader); each window's records are cut into CIGAR ranges on the
// device (hbam_summarize_ranges) and nextKeyValue() hands out (LongWritable key, Range) exactly in
// the reference's order, raising its exception (the base reader's, IllegalArgumentException for a
// CIGAR op code > 8, IndexOutOfBoundsException for a mapped record without a range) where it does.
// Lives in the chipster package because Range is package-private there.  Source only (no JDK).
package org.seqdoop.hadoop_bam.cli.plugins.chipster;

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

import htsjdk.samtools.SAMFileHeader;
import htsjdk.samtools.util.RuntimeIOException;

import hbparquet.hadoop.util.ContextUtil;
import org.seqdoop.hadoop_bam.FileVirtualSplit;
import org.seqdoop.hadoop_bam.hip.Hbam;
import org.seqdoop.hadoop_bam.hip.HipBAMRecordReader;
import org.seqdoop.hadoop_bam.hip.SplitSource;
import org.seqdoop.hadoop_bam.util.SAMHeaderReader;

public class HipSummarizeRecordReader extends RecordReader<LongWritable, Range> {
  private final LongWritable key = new LongWritable();
  private final Range value = new Range();

  private Hbam hbam;
  private SplitSource source;
  private Arena arena, window;       // reader lifetime / the current window's host copies
  private MemorySegment stream, dev, ranges;
  private MemorySegment keys, begs, ends, revs;
  private long n, i;
  private int status;
  private boolean last;

  @Override public void initialize(InputSplit spl, TaskAttemptContext ctx) throws IOException {
    final Configuration conf = ContextUtil.getConfiguration(ctx);
    final FileVirtualSplit split = (FileVirtualSplit) spl;
    final Path file = split.getPath();
    final FileSystem fs = file.getFileSystem(conf);
    final SAMFileHeader header;
    try (FSDataInputStream in = fs.open(file)) {
      header = SAMHeaderReader.readSAMHeaderFrom(in, conf);
    }
    final long len = fs.getFileStatus(file).getLen();
    arena = Arena.ofShared();
    hbam = new Hbam(conf.getInt(HipBAMRecordReader.DEVICE_PROPERTY, 0), false);
    source = new SplitSource(fs, file, arena);  // the split's bytes only (positioned reads)
    stream = source.open(hbam, len, split.getStartVirtualOffset(), split.getEndVirtualOffset(),
                         header.getSequenceDictionary().size(),
                         conf.getLong(HipBAMRecordReader.WINDOW_BYTES_PROPERTY, 1L << 30));
    dev = arena.allocate(Hbam.COLUMNS);
    ranges = arena.allocate(Hbam.RANGES);
    n = i = 0;
    status = Hbam.OK;
    last = false;
  }

  private static long off(String f) {
    return Hbam.RANGES.byteOffset(MemoryLayout.PathElement.groupElement(f));
  }

  /** hbam_split_next + hbam_summarize_ranges + downloads of the window's ranges. */
  private boolean nextWindow() {
    try {
      final int rc = (int) Hbam.SPLIT_NEXT.invokeExact(stream, dev);
      if (rc < 0) throw new RuntimeIOException("hbam_split_next: " + hbam.lastError());
      if (rc == 0) { last = true; return false; }
      final int rc2 = (int) Hbam.SUMMARIZE.invokeExact(hbam.context(), dev, ranges);
      if (rc2 != Hbam.OK) throw new RuntimeIOException("hbam_summarize_ranges: " + hbam.lastError());
    } catch (RuntimeException e) {
      throw e;
    } catch (Throwable t) {
      throw new RuntimeIOException(t);
    }
    if (window != null) window.close();
    window = Arena.ofConfined();
    n = ranges.get(ValueLayout.JAVA_LONG, off("n"));
    status = ranges.get(ValueLayout.JAVA_INT, off("status"));
    if (status != Hbam.OK) last = true;
    keys = hbam.download(ranges.get(ValueLayout.ADDRESS, off("key")), 8 * n, window);
    begs = hbam.download(ranges.get(ValueLayout.ADDRESS, off("beg")), 4 * n, window);
    ends = hbam.download(ranges.get(ValueLayout.ADDRESS, off("end")), 4 * n, window);
    revs = hbam.download(ranges.get(ValueLayout.ADDRESS, off("rev")), n, window);
    i = 0;
    return true;
  }

  @Override public boolean nextKeyValue() {
    while (i >= n) {
      if (status != Hbam.OK) {
        final int s = status;
        status = Hbam.OK;
        throw Hbam.exceptionFor(s, "SummarizeRecordReader.nextKeyValue");
      }
      if (last || !nextWindow()) return false;
    }
    key.set(keys.getAtIndex(ValueLayout.JAVA_LONG, i));
    value.beg.set(begs.getAtIndex(ValueLayout.JAVA_INT, i));
    value.end.set(ends.getAtIndex(ValueLayout.JAVA_INT, i));
    value.reverseStrand.set(revs.get(ValueLayout.JAVA_BYTE, i) != 0);
    ++i;
    return true;
  }

  @Override public LongWritable getCurrentKey() { return key; }
  @Override public Range getCurrentValue() { return value; }
  @Override public float getProgress() { return last && i >= n ? 1 : 0; }

  @Override public void close() throws IOException {
    try {
      if (stream != null && stream.address() != 0) Hbam.SPLIT_CLOSE.invokeExact(stream);
      if (source != null) source.close();
    } catch (Throwable t) {
      throw new IOException(t);
    } finally {
      stream = null;
      source = null;
      if (window != null) window.close();
      window = null;
      if (hbam != null) hbam.close();
      hbam = null;
      if (arena != null) arena.close();
      arena = null;
    }
  }
}
