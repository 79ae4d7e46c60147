// Drop-in body of org.seqdoop.hadoop_bam.BCFSplitGuesser (BCFSplitGuesser.java:52-455) over the C
// ABI: the header is read by hbam_bcf_parse_header (BCF2Codec.readHeader's counts, :105-112);
// guessNextBCFRecordStart buffers the window the reference buffers (:133-145: min((int)(end-beg),
// 2*0xffff+0xfffe) bytes for BGZF, 0x80000 uncompressed, cut at the end of the stream) and hands
// it to hbam_guess_bcf_windows, which runs the reference's state machine (k_guess_bcf).
package org.seqdoop.hadoop_bam.hip;

import java.io.IOException;
import java.io.InputStream;
import java.lang.foreign.*;

import htsjdk.samtools.seekablestream.SeekableStream;

public class HipBCFSplitGuesser {
  private final SeekableStream inFile;
  private final Hbam hbam;
  private final MemorySegment header;  // hbam_bcf_header (global arena: lives with the guesser)
  private final boolean bgzf;

  public HipBCFSplitGuesser(SeekableStream ss) throws IOException {
    this(ss, ss);
  }

  public HipBCFSplitGuesser(SeekableStream ss, InputStream headerStream) throws IOException {
    inFile = ss;
    hbam = HipBAMRecordReader.context(null);
    header = Arena.ofAuto().allocate(Hbam.BCF_HEADER);
    byte[] head = headerStream.readNBytes(1 << 20);
    final byte[] magic = Hbam.readWindow(ss, 0, 18);
    for (;;) {  // a header longer than the prefix (HBAM_EMORE, e.g. many samples): read 4x more
      int rc;
      try (Arena a = Arena.ofConfined()) {
        final MemorySegment h = a.allocate(Math.max(head.length, 1));
        MemorySegment.copy(head, 0, h, ValueLayout.JAVA_BYTE, 0, head.length);
        rc = (int) Hbam.BCF_PARSE_HEADER.invokeExact(hbam.context(), h, (long) head.length, header);
      } catch (RuntimeException e) {
        throw e;
      } catch (Throwable t) {
        throw new IOException(t);
      }
      if (rc == Hbam.EMORE) {
        final byte[] more = headerStream.readNBytes(3 * head.length);
        if (more.length > 0) {
          final byte[] grown = java.util.Arrays.copyOf(head, head.length + more.length);
          System.arraycopy(more, 0, grown, head.length, more.length);
          head = grown;
          continue;
        }
      }
      if (rc != Hbam.OK) throw Hbam.exceptionFor(rc, "BCF2Codec.readHeader: " + hbam.lastError());
      break;
    }
    // BlockCompressedInputStream.isValidFile on the data stream (:99-103): the 16 header bytes
    // hbam_bcf_parse_header and the mirror check (ID1 ID2 CM FLG, XLEN = 6, 'B' 'C', SLEN = 2)
    bgzf = magic.length == 18 && (magic[0] & 0xff) == 0x1f && (magic[1] & 0xff) == 0x8b && magic[2] == 8
        && magic[3] == 4 && magic[10] == 6 && magic[11] == 0 && magic[12] == 'B' && magic[13] == 'C'
        && magic[14] == 2 && magic[15] == 0;
    header.set(ValueLayout.JAVA_INT, 12, bgzf ? 1 : 0);
  }

  public boolean isBGZF() { return bgzf; }

  /** Finds a (virtual in the case of BGZF) BCF record position in [beg,end); end if none. */
  public long guessNextBCFRecordStart(long beg, long end) throws IOException {
    final long fileLen = inFile.length();
    final long n;
    try {
      n = (long) Hbam.GUESS_BCF_WINDOW_LEN.invokeExact(fileLen, beg, end, bgzf ? 1 : 0);
    } catch (Throwable t) {
      throw new IOException(t);
    }
    final byte[] w = n > 0 ? Hbam.readWindow(inFile, beg, (int) n) : new byte[0];
    if (w.length != n) throw new IOException("short read of a guess window at " + beg);
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment ws = a.allocate(Math.max(w.length, 1));
      MemorySegment.copy(w, 0, ws, ValueLayout.JAVA_BYTE, 0, w.length);
      final MemorySegment off = a.allocateFrom(ValueLayout.JAVA_LONG, 0L, n);
      final MemorySegment b = a.allocateFrom(ValueLayout.JAVA_LONG, beg), e = a.allocateFrom(ValueLayout.JAVA_LONG, end);
      final MemorySegment out = a.allocate(ValueLayout.JAVA_LONG), err = a.allocate(ValueLayout.JAVA_INT);
      final int rc = (int) Hbam.GUESS_BCF_WINDOWS.invokeExact(hbam.context(), ws, 0, off, fileLen, b, e, 1L,
                                                            header, out, err);
      if (rc != Hbam.OK) throw new IOException("hbam_guess_bcf_windows: " + hbam.lastError());
      final int ex = err.get(ValueLayout.JAVA_INT, 0);
      if (ex != Hbam.OK)  // an exception the reference lets escape (:258-273)
        throw Hbam.exceptionFor(ex, "guessNextBCFRecordStart(" + beg + ", " + end + ")");
      return out.get(ValueLayout.JAVA_LONG, 0);
    } catch (IOException | RuntimeException ex) {
      throw ex;
    } catch (Throwable t) {
      throw new IOException(t);
    }
  }

  MemorySegment header() { return header; }
}
