// Drop-in body of the Sort plugin's SortRecordReader (cli/plugins/Sort.java:254-295) over the
// GPU reader: when the inputs' sequence dictionaries differ, Utils.correctSAMRecordForMerging
// (cli/Utils.java:286-313) runs on the device over every window of decoded records
// (hbam_merge_remap: refID / mate refID onto the merged dictionary, the key recomputed where
// refID changed), so the keys HipBAMRecordReader hands out are already SortRecordReader's.
// The merged dictionary is htsjdk's own (Utils.getSAMHeaderMerger).
package org.seqdoop.hadoop_bam.hip;

import java.io.IOException;

import org.apache.hadoop.conf.Configuration;
import org.apache.hadoop.io.LongWritable;
import org.apache.hadoop.mapreduce.InputSplit;
import org.apache.hadoop.mapreduce.RecordReader;
import org.apache.hadoop.mapreduce.TaskAttemptContext;

import htsjdk.samtools.SAMFileHeader;
import htsjdk.samtools.SamFileHeaderMerger;

import hbparquet.hadoop.util.ContextUtil;
import org.seqdoop.hadoop_bam.SAMRecordWritable;
import org.seqdoop.hadoop_bam.cli.Utils;

public class HipSortRecordReader extends RecordReader<LongWritable, SAMRecordWritable> {
  private final HipBAMRecordReader baseRR = new HipBAMRecordReader();

  @Override public void initialize(InputSplit spl, TaskAttemptContext ctx) throws IOException {
    final Configuration conf = ContextUtil.getConfiguration(ctx);
    baseRR.initialize(spl, ctx);
    final SamFileHeaderMerger merger = Utils.getSAMHeaderMerger(conf);
    if (merger.hasMergedSequenceDictionary()) {
      final SAMFileHeader h = baseRR.header();
      final int n = h.getSequenceDictionary().size();
      final int[] map = new int[n];
      for (int i = 0; i < n; ++i) map[i] = merger.getMergedSequenceIndex(h, i);
      baseRR.setMergeMap(map);
    }
    // RG / PG collisions (Utils.java:314-323) are not remapped on the device: such jobs keep
    // the reference's SortRecordReader.
    if (merger.hasReadGroupCollisions() || merger.hasProgramGroupCollisions())
      throw new IOException("read / program group collisions: use the reference SortRecordReader");
  }

  @Override public boolean nextKeyValue() { return baseRR.nextKeyValue(); }
  @Override public LongWritable getCurrentKey() { return baseRR.getCurrentKey(); }
  @Override public SAMRecordWritable getCurrentValue() { return baseRR.getCurrentValue(); }
  @Override public float getProgress() { return baseRR.getProgress(); }
  @Override public void close() throws IOException { baseRR.close(); }
}
