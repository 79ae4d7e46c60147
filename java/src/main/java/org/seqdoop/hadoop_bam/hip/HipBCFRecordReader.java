// Drop-in body of org.seqdoop.hadoop_bam.BCFRecordReader (BCFRecordReader.java:52-175) over the C
// ABI.  initialize() maps the split's bytes from its start to 1 MiB past vEnd's block (a BGZF split
// reads through BGZFLimitingStream, :177-237, which stops in a block starting exactly at the split
// end; while it runs past the window, HBAM_EMORE, the window grows 4x, up to the end of the file;
// an uncompressed split reads to the end of the file) and hbam_bcf_decode_split decodes every
// record on the device, inflating only the blocks the stream reaches; nextKeyValue hands out
// the key (contig index << 32 | start - 1, :167-171) and raises, after the last record, the
// exception the reference's BCF2Codec.decode raises there.  getCurrentValue() exposes the raw
// BCF2 record bytes and the decoded site fields (a VariantContext is built by the caller's
// htsjdk from those bytes when it needs one).
package org.seqdoop.hadoop_bam.hip;

import java.io.IOException;
import java.lang.foreign.*;
import java.nio.channels.FileChannel;
import java.nio.file.Path;
import java.nio.file.StandardOpenOption;

import org.apache.hadoop.io.LongWritable;
import org.apache.hadoop.mapreduce.InputSplit;
import org.apache.hadoop.mapreduce.RecordReader;
import org.apache.hadoop.mapreduce.TaskAttemptContext;
import org.apache.hadoop.mapreduce.lib.input.FileSplit;

import org.seqdoop.hadoop_bam.FileVirtualSplit;

public class HipBCFRecordReader extends RecordReader<LongWritable, HipBCFRecordReader.Record> {
  /** One decoded record: site fields and its BCF2 bytes (l_shared | l_indiv | site | genotypes). */
  public static final class Record {
    public int contig, pos0, rlen, nAlleleInfo, nFmtSample;
    public float qual;
    public byte[] bytes;
  }

  private final LongWritable key = new LongWritable();
  private final Record value = new Record();
  private Arena arena;
  private long n, i;
  private int status;
  private MemorySegment keys, chrom, pos, rlen, qual, nai, nfs, recOff, lshared, lindiv, data;

  @Override public void initialize(InputSplit spl, TaskAttemptContext ctx) throws IOException {
    final Hbam hbam = HipBAMRecordReader.context(ctx.getConfiguration());
    final boolean virt = spl instanceof FileVirtualSplit;
    final Path path = Path.of((virt ? ((FileVirtualSplit) spl).getPath() : ((FileSplit) spl).getPath())
                                  .toUri().getPath());
    arena = Arena.ofConfined();
    try (FileChannel ch = FileChannel.open(path, StandardOpenOption.READ)) {
      final long fileLen = ch.size();
      final MemorySegment h = arena.allocate(Hbam.BCF_HEADER);
      int rc;
      for (long want = 1 << 20; ; want *= 4) {  // a header longer than the prefix: HBAM_EMORE, read more
        final MemorySegment head = ch.map(FileChannel.MapMode.READ_ONLY, 0, Math.min(fileLen, want), arena);
        rc = (int) Hbam.BCF_PARSE_HEADER.invokeExact(hbam.context(), head, head.byteSize(), h);
        if (rc != Hbam.EMORE || want >= fileLen) break;
      }
      if (rc != Hbam.OK) throw new IOException("BCF2Codec.readHeader: " + hbam.lastError());
      final long start, end, base;
      if (virt) {
        start = ((FileVirtualSplit) spl).getStartVirtualOffset();
        end = ((FileVirtualSplit) spl).getEndVirtualOffset();
        base = start >>> 16;
      } else {
        start = ((FileSplit) spl).getStart();
        end = ((FileSplit) spl).getLength();
        base = Math.min(Math.max(start, h.get(ValueLayout.JAVA_LONG, 16)), fileLen);
      }
      final boolean bgzf = h.get(ValueLayout.JAVA_INT, 12) != 0;
      final MemorySegment cols = arena.allocate(Hbam.BCF_COLUMNS);
      for (long tail = 1 << 20; ; tail *= 4) {
        final long stop = !bgzf ? fileLen : Math.min(fileLen, (end >>> 16) + tail);
        final MemorySegment win = ch.map(FileChannel.MapMode.READ_ONLY, base, stop - base, arena);
        rc = (int) Hbam.BCF_DECODE_SPLIT.invokeExact(hbam.context(), win, 0, base, stop - base, fileLen, h,
                                                     start, end, cols);
        if (rc != Hbam.OK) throw new IOException("hbam_bcf_decode_split: " + hbam.lastError());
        status = cols.get(ValueLayout.JAVA_INT, 8);
        if (status != Hbam.EMORE || stop == fileLen) break;
      }
      n = cols.get(ValueLayout.JAVA_LONG, 0);
      keys = down(hbam, cols, "key", 8);
      chrom = down(hbam, cols, "chrom", 4);
      pos = down(hbam, cols, "pos", 4);
      rlen = down(hbam, cols, "rlen", 4);
      qual = down(hbam, cols, "qual", 4);
      nai = down(hbam, cols, "n_allele_info", 4);
      nfs = down(hbam, cols, "n_fmt_sample", 4);
      recOff = down(hbam, cols, "rec_off", 8);
      lshared = down(hbam, cols, "l_shared", 4);
      lindiv = down(hbam, cols, "l_indiv", 4);
      final long dl = cols.get(ValueLayout.JAVA_LONG, Hbam.BCF_COLUMNS.byteOffset(
          MemoryLayout.PathElement.groupElement("data_len")));
      data = hbam.download(ptr(cols, "data"), dl, arena);
    } catch (IOException | RuntimeException e) {
      throw e;
    } catch (Throwable t) {
      throw new IOException(t);
    }
    i = 0;
  }

  private static MemorySegment ptr(MemorySegment cols, String f) {
    return cols.get(ValueLayout.ADDRESS, Hbam.BCF_COLUMNS.byteOffset(MemoryLayout.PathElement.groupElement(f)));
  }

  private MemorySegment down(Hbam hbam, MemorySegment cols, String f, int w) {
    return hbam.download(ptr(cols, f), n * w, arena);
  }

  @Override public boolean nextKeyValue() {
    if (i >= n) {
      if (status != Hbam.OK) throw Hbam.exceptionFor(status, "BCFRecordReader.nextKeyValue");
      return false;
    }
    key.set(keys.getAtIndex(ValueLayout.JAVA_LONG, i));
    value.contig = chrom.getAtIndex(ValueLayout.JAVA_INT, i);
    value.pos0 = pos.getAtIndex(ValueLayout.JAVA_INT, i);
    value.rlen = rlen.getAtIndex(ValueLayout.JAVA_INT, i);
    value.qual = Float.intBitsToFloat(qual.getAtIndex(ValueLayout.JAVA_INT, i));
    value.nAlleleInfo = nai.getAtIndex(ValueLayout.JAVA_INT, i);
    value.nFmtSample = nfs.getAtIndex(ValueLayout.JAVA_INT, i);
    final long o = recOff.getAtIndex(ValueLayout.JAVA_LONG, i);
    final int len = 8 + lshared.getAtIndex(ValueLayout.JAVA_INT, i) + lindiv.getAtIndex(ValueLayout.JAVA_INT, i);
    value.bytes = data.asSlice(o, len).toArray(ValueLayout.JAVA_BYTE);
    ++i;
    return true;
  }

  @Override public LongWritable getCurrentKey() { return key; }
  @Override public Record getCurrentValue() { return value; }
  @Override public float getProgress() { return n == 0 ? 1 : (float) i / n; }
  @Override public void close() { if (arena != null) arena.close(); arena = null; }
}
