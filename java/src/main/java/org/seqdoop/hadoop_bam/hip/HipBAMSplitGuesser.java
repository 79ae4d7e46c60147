// Drop-in body of org.seqdoop.hadoop_bam.BAMSplitGuesser (BAMSplitGuesser.java:50-398) over the
// C ABI: the constructors read the header exactly as the reference does (SAMHeaderReader over
// the header stream, :94-103, and the magic check of :77-88); guessNextBAMRecordStart buffers
// the window the reference buffers (:114-125: min((int)(end-beg), 262139) bytes at beg, cut at
// the end of the stream) and hands it to hbam_guess_windows, which runs the reference's state
// machine for it on one GPU wave.  guessNextBAMRecordStarts(beg[], end[]) is the batched form
// HipBAMInputFormat uses: every FileSplit's window in one device call.
package org.seqdoop.hadoop_bam.hip;

import java.io.IOException;
import java.io.InputStream;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;

import org.apache.hadoop.conf.Configuration;

import htsjdk.samtools.SAMFormatException;
import htsjdk.samtools.seekablestream.SeekableStream;

import org.seqdoop.hadoop_bam.util.SAMHeaderReader;

public class HipBAMSplitGuesser {
  private static final int BGZF_MAGIC = 0x04088b1f;

  private final SeekableStream inFile;
  private final int referenceSequenceCount;
  private final Hbam hbam;

  /** The stream must point to a valid BAM file, because the header is read from it. */
  public HipBAMSplitGuesser(SeekableStream ss, Configuration conf) throws IOException {
    this(ss, ss, conf);
    // secondary check that the header points to a BAM file (:83-87)
    final ByteBuffer buf = ByteBuffer.allocate(4).order(ByteOrder.LITTLE_ENDIAN);
    ss.seek(0);
    if (ss.read(buf.array(), 0, 4) != 4 || buf.getInt(0) != BGZF_MAGIC)
      throw new SAMFormatException("Does not seem like a BAM file");
  }

  public HipBAMSplitGuesser(SeekableStream ss, InputStream headerStream, Configuration conf)
      throws IOException {
    inFile = ss;
    referenceSequenceCount =
        SAMHeaderReader.readSAMHeaderFrom(headerStream, conf).getSequenceDictionary().size();
    hbam = HipBAMRecordReader.context(conf);
  }

  /** Finds a virtual BAM record position in the physical position range [beg,end). Returns end
   *  if no BAM record was found. */
  public long guessNextBAMRecordStart(long beg, long end) throws IOException {
    return guessNextBAMRecordStarts(new long[] {beg}, new long[] {end})[0];
  }

  /** guessNextBAMRecordStart for k ranges in one device call (each guess independent, as k
   *  calls of the reference's method: only windows shorter than 4 bytes could see the 8-byte
   *  buffer a previous call left, and those return `end`). */
  public long[] guessNextBAMRecordStarts(long[] beg, long[] end) throws IOException {
    final int k = beg.length;
    final long fileLen = inFile.length();
    final long[] off = new long[k + 1];
    final byte[][] w = new byte[k][];
    for (int i = 0; i < k; ++i) {
      final long n = Hbam.guessWindowLen(fileLen, beg[i], end[i]);
      w[i] = n > 0 ? Hbam.readWindow(inFile, beg[i], (int) n) : new byte[0];
      if (w[i].length != n) throw new IOException("short read of a guess window at " + beg[i]);
      off[i + 1] = off[i] + n;
    }
    final byte[] all = new byte[(int) off[k]];
    for (int i = 0; i < k; ++i) System.arraycopy(w[i], 0, all, (int) off[i], w[i].length);
    final long[] out = new long[k];
    final int[] err = new int[k];
    hbam.guessWindows(all, off, fileLen, beg, end, referenceSequenceCount, out, err);
    for (int i = 0; i < k; ++i)
      if (err[i] != Hbam.OK)  // an exception the reference lets escape (:144-152, :194-207)
        throw Hbam.exceptionFor(err[i], "guessNextBAMRecordStart(" + beg[i] + ", " + end[i] + ")");
    return out;
  }
}
