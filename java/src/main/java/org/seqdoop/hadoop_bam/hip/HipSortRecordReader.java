// Drop-in body of the Sort plugin's SortRecordReader (cli/plugins/Sort.java:254-295) over the
// GPU reader: when the inputs' sequence dictionaries differ, Utils.correctSAMRecordForMerging
// (cli/Utils.java:286-313) runs on the device over every window of decoded records
// (hbam_merge_remap: refID / mate refID onto the merged dictionary, the key recomputed where
// refID changed), so the keys HipBAMRecordReader hands out are already SortRecordReader's; with
// read- / program-group ID collisions the PG / RG tags are rewritten and the records re-encoded
// there too (hbam_rewrite_groups).  The merger is htsjdk's own (Utils.getSAMHeaderMerger).
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
    // RG / PG collisions (Utils.java:314-324): both tags translated through htsjdk's program-group
    // table (the reference's getProgramGroupId for RG too), on the device (hbam_rewrite_groups)
    if (merger.hasReadGroupCollisions() || merger.hasProgramGroupCollisions())
      baseRR.setGroupTable(groupTable(merger, baseRR.header()));
  }

  /** hbam_rewrite_groups' table (include/hbam.h): for PG then RG, u8 mode, u16 count, entries
   *  {u16 len, old id, i16 len, merged id}: getProgramGroupId(h, id) of every @PG id of h (an id
   *  missing from the table, and any other value, is removed: get() == null); mode 2 when h has no
   *  translation table (the reference's NullPointerException). */
  static byte[] groupTable(SamFileHeaderMerger merger, SAMFileHeader h) throws IOException {
    final java.io.ByteArrayOutputStream out = new java.io.ByteArrayOutputStream();
    final java.util.List<htsjdk.samtools.SAMProgramRecord> pgs = h.getProgramRecords();
    boolean table = true;
    try {
      merger.getProgramGroupId(h, pgs.isEmpty() ? "" : pgs.get(0).getId());
    } catch (NullPointerException e) {
      table = false;
    }
    for (boolean collides : new boolean[] {merger.hasProgramGroupCollisions(), merger.hasReadGroupCollisions()}) {
      final int mode = !collides ? 0 : table ? 1 : 2;
      final java.util.List<htsjdk.samtools.SAMProgramRecord> es = mode == 1 ? pgs : java.util.Collections.emptyList();
      out.write(mode);
      out.write(es.size() & 0xff);
      out.write((es.size() >> 8) & 0xff);
      for (htsjdk.samtools.SAMProgramRecord pg : es) {
        final byte[] o = pg.getId().getBytes(java.nio.charset.StandardCharsets.ISO_8859_1);
        final String nw = merger.getProgramGroupId(h, pg.getId());
        final byte[] w = nw == null ? new byte[0] : nw.getBytes(java.nio.charset.StandardCharsets.ISO_8859_1);
        final int wl = nw == null ? -1 : w.length;
        out.write(o.length & 0xff);
        out.write((o.length >> 8) & 0xff);
        out.write(o);
        out.write(wl & 0xff);
        out.write((wl >> 8) & 0xff);
        out.write(w);
      }
    }
    return out.toByteArray();
  }

  @Override public boolean nextKeyValue() { return baseRR.nextKeyValue(); }
  @Override public LongWritable getCurrentKey() { return baseRR.getCurrentKey(); }
  @Override public SAMRecordWritable getCurrentValue() { return baseRR.getCurrentValue(); }
  @Override public float getProgress() { return baseRR.getProgress(); }
  @Override public void close() throws IOException { baseRR.close(); }
}
