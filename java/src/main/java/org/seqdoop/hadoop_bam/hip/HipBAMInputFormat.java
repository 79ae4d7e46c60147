// Drop-in body of org.seqdoop.hadoop_bam.BAMInputFormat (BAMInputFormat.java:50-229) whose
// split side runs on the GPU: getSplits keeps the reference's order and rules (sort by path,
// indexed splits from a .splitting-bai when present, else probabilistic splits), and
// addProbabilisticSplits guesses every FileSplit of a file in ONE device call
// (HipBAMSplitGuesser.guessNextBAMRecordStarts -> hbam_guess_windows: only the header and each
// split's guess window are read from the file), then applies the reference's merge loop
// (:181-222) to the guesses.  Records are read by HipBAMRecordReader.
package org.seqdoop.hadoop_bam.hip;

import java.io.IOException;
import java.util.ArrayList;
import java.util.Collections;
import java.util.Comparator;
import java.util.List;

import org.apache.hadoop.conf.Configuration;
import org.apache.hadoop.fs.Path;
import org.apache.hadoop.io.LongWritable;
import org.apache.hadoop.mapreduce.InputSplit;
import org.apache.hadoop.mapreduce.JobContext;
import org.apache.hadoop.mapreduce.RecordReader;
import org.apache.hadoop.mapreduce.TaskAttemptContext;
import org.apache.hadoop.mapreduce.lib.input.FileInputFormat;
import org.apache.hadoop.mapreduce.lib.input.FileSplit;

import htsjdk.samtools.seekablestream.SeekableStream;

import hbparquet.hadoop.util.ContextUtil;
import org.seqdoop.hadoop_bam.FileVirtualSplit;
import org.seqdoop.hadoop_bam.SAMRecordWritable;
import org.seqdoop.hadoop_bam.SplittingBAMIndex;
import org.seqdoop.hadoop_bam.util.WrapSeekable;

public class HipBAMInputFormat extends FileInputFormat<LongWritable, SAMRecordWritable> {
  private Path getIdxPath(Path path) { return path.suffix(".splitting-bai"); }

  @Override public RecordReader<LongWritable, SAMRecordWritable> createRecordReader(
      InputSplit split, TaskAttemptContext ctx) throws InterruptedException, IOException {
    final RecordReader<LongWritable, SAMRecordWritable> rr = new HipBAMRecordReader();
    rr.initialize(split, ctx);
    return rr;
  }

  @Override public List<InputSplit> getSplits(JobContext job) throws IOException {
    return getSplits(super.getSplits(job), ContextUtil.getConfiguration(job));
  }

  public List<InputSplit> getSplits(List<InputSplit> splits, Configuration cfg) throws IOException {
    Collections.sort(splits, new Comparator<InputSplit>() {  // :84-90
      public int compare(InputSplit a, InputSplit b) {
        return ((FileSplit) a).getPath().compareTo(((FileSplit) b).getPath());
      }
    });
    final List<InputSplit> newSplits = new ArrayList<InputSplit>(splits.size());
    for (int i = 0; i < splits.size();) {
      try {
        i = addIndexedSplits(splits, i, newSplits, cfg);
      } catch (IOException e) {
        i = addProbabilisticSplits(splits, i, newSplits, cfg);
      }
    }
    return newSplits;
  }

  // :107-159 (the index gives exact starts; no guessing)
  private int addIndexedSplits(List<InputSplit> splits, int i, List<InputSplit> newSplits,
                               Configuration cfg) throws IOException {
    final Path file = ((FileSplit) splits.get(i)).getPath();
    final List<InputSplit> potential = new ArrayList<InputSplit>();
    final SplittingBAMIndex idx = new SplittingBAMIndex(file.getFileSystem(cfg).open(getIdxPath(file)));
    int splitsEnd = splits.size();
    for (int j = i; j < splitsEnd; ++j)
      if (!file.equals(((FileSplit) splits.get(j)).getPath())) splitsEnd = j;
    for (int j = i; j < splitsEnd; ++j) {
      final FileSplit fs = (FileSplit) splits.get(j);
      final long start = fs.getStart(), end = start + fs.getLength();
      final Long blockStart = idx.nextAlignment(start);
      final Long blockEnd = j == splitsEnd - 1 ? idx.prevAlignment(end) | 0xffff : idx.nextAlignment(end);
      if (blockStart == null || blockEnd == null) return addProbabilisticSplits(splits, i, newSplits, cfg);
      potential.add(new FileVirtualSplit(file, blockStart, blockEnd, fs.getLocations()));
    }
    newSplits.addAll(potential);
    return splitsEnd;
  }

  // :163-224 with the guesses batched
  private int addProbabilisticSplits(List<InputSplit> splits, int i, List<InputSplit> newSplits,
                                     Configuration cfg) throws IOException {
    final Path path = ((FileSplit) splits.get(i)).getPath();
    final SeekableStream sin = WrapSeekable.openPath(path.getFileSystem(cfg), path);
    final HipBAMSplitGuesser guesser = new HipBAMSplitGuesser(sin, cfg);
    int j = i;
    while (j < splits.size() && ((FileSplit) splits.get(j)).getPath().equals(path)) ++j;
    final long[] beg = new long[j - i], end = new long[j - i];
    for (int q = i; q < j; ++q) {
      final FileSplit f = (FileSplit) splits.get(q);
      beg[q - i] = f.getStart();
      end[q - i] = f.getStart() + f.getLength();
    }
    final long[] guess = guesser.guessNextBAMRecordStarts(beg, end);
    FileVirtualSplit previousSplit = null;
    for (int q = i; q < j; ++q) {
      final long alignedBeg = guess[q - i];
      final long alignedEnd = end[q - i] << 16 | 0xffff;
      if (alignedBeg == end[q - i]) {
        if (previousSplit == null)
          throw new IOException("'" + path + "': no reads in first split: bad BAM file or tiny split size?");
        previousSplit.setEndVirtualOffset(alignedEnd);
      } else {
        previousSplit = new FileVirtualSplit(path, alignedBeg, alignedEnd,
                                             ((FileSplit) splits.get(q)).getLocations());
        newSplits.add(previousSplit);
      }
    }
    sin.close();
    return j;
  }

  @Override public boolean isSplitable(JobContext job, Path path) { return true; }
}
