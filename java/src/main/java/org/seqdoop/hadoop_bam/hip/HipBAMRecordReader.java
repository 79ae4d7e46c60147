// Drop-in body of org.seqdoop.hadoop_bam.BAMRecordReader (BAMRecordReader.java:48-188) over
// the C ABI: initialize() decodes the whole FileVirtualSplit on the GPU (hbam_decode_split),
// nextKeyValue() hands out (LongWritable key, SAMRecordWritable) from the columns and throws
// the reference's exception at the record where the reference would.
package org.seqdoop.hadoop_bam.hip;

import java.io.IOException;
import java.lang.foreign.*;

import org.apache.hadoop.io.LongWritable;
import org.apache.hadoop.mapreduce.InputSplit;
import org.apache.hadoop.mapreduce.RecordReader;
import org.apache.hadoop.mapreduce.TaskAttemptContext;

import htsjdk.samtools.BAMRecordCodec;
import htsjdk.samtools.SAMFileHeader;
import htsjdk.samtools.SAMRecord;

import org.seqdoop.hadoop_bam.FileVirtualSplit;
import org.seqdoop.hadoop_bam.LazyBAMRecordFactory;
import org.seqdoop.hadoop_bam.SAMRecordWritable;

public class HipBAMRecordReader extends RecordReader<LongWritable, SAMRecordWritable> {
  private final LongWritable key = new LongWritable();
  private final SAMRecordWritable record = new SAMRecordWritable();
  private Arena arena;
  private MemorySegment host;          // hbam_columns (host copy)
  private long n, i;
  private int status;
  private MemorySegment keys, recOff, blockSize, ubuf;
  private SAMFileHeader header;

  @Override public void initialize(InputSplit spl, TaskAttemptContext ctx) throws IOException {
    final FileVirtualSplit split = (FileVirtualSplit) spl;
    // (1) map the file (HDFS -> pinned host buffer) and read the header as the reference does
    // (2) hbam_decode_split(ctx, buf, 0, 0, len, len, vStart, vEnd, n_ref, &dev)
    // (3) hbam_columns_to_host(ctx, &dev, &host); keep key/rec_off/block_size/ubuf views
    // The payload bytes of record i are ubuf[rec_off[i] .. rec_off[i]+4+block_size[i]):
    // exactly what BAMRecordCodec.decode() reads, so SAMRecordWritable gets a lazily
    // decoded BAMRecord built by LazyBAMRecordFactory from those bytes.
    throw new UnsupportedOperationException("reference shim: see INTEGRATION.md");
  }

  @Override public boolean nextKeyValue() {
    if (i >= n) {
      if (status != Hbam.OK && i == n) { ++i; throw Hbam.exceptionFor(status, "record " + n); }
      return false;
    }
    key.set(keys.getAtIndex(ValueLayout.JAVA_LONG, i));
    // record.set(decodeLazy(ubuf, recOff[i], blockSize[i])) — BAMRecordCodec over a
    // ByteArrayInputStream of the record bytes, header attached (BAMRecordReader.java:176-186)
    ++i;
    return true;
  }

  @Override public LongWritable getCurrentKey() { return key; }
  @Override public SAMRecordWritable getCurrentValue() { return record; }
  @Override public float getProgress() { return n == 0 ? 1 : (float) i / n; }
  @Override public void close() { if (arena != null) arena.close(); }
}
