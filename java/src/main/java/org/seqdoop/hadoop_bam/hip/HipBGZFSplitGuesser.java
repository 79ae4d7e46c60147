// Drop-in body of org.seqdoop.hadoop_bam.util.BGZFSplitGuesser (util/BGZFSplitGuesser.java:
// 30-148): guessNextBGZFBlockStart reads the one window the reference reads (:62-63,
// min((int)(end-beg), 131069) bytes at beg) and hands it to hbam_guess_bgzf_window.
package org.seqdoop.hadoop_bam.hip;

import java.io.IOException;
import java.lang.foreign.*;

import org.apache.hadoop.conf.Configuration;
import org.apache.hadoop.fs.FSDataInputStream;

import org.seqdoop.hadoop_bam.util.WrapSeekable;

public class HipBGZFSplitGuesser {
  private final FSDataInputStream inFile;
  private final long fileLen;
  private final Hbam hbam;

  public HipBGZFSplitGuesser(FSDataInputStream is, long fileLen, Configuration conf) throws IOException {
    inFile = is;
    this.fileLen = fileLen;
    hbam = HipBAMRecordReader.context(conf);
  }

  public long guessNextBGZFBlockStart(long beg, long end) throws IOException {
    final int n = (int) Hbam.guessBgzfWindowLen(fileLen, beg, end);
    final byte[] w = new byte[n];
    inFile.seek(beg);
    int got = 0;
    if (n > 0) {  // ONE read() call, as the reference (:62-63)
      final int r = inFile.read(w, 0, n);
      got = Math.max(r, 0);
    }
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment seg = a.allocate(Math.max(got, 1));
      MemorySegment.copy(w, 0, seg, ValueLayout.JAVA_BYTE, 0, got);
      final MemorySegment err = a.allocate(ValueLayout.JAVA_INT);
      // a short read leaves the window shorter than the file would give: pass the bytes held
      // as the file's extent so the guesser sees exactly them
      final long extent = got == n ? fileLen : beg + got;
      final long r = (long) Hbam.GUESS_BGZF_WINDOW.invokeExact(hbam.context(), seg, 0, (long) got, extent,
                                                             beg, end, err);
      final int e = err.get(ValueLayout.JAVA_INT, 0);
      if (e != Hbam.OK) throw new IOException("guessNextBGZFBlockStart: " + hbam.lastError());
      return r;
    } catch (IOException | RuntimeException ex) {
      throw ex;
    } catch (Throwable t) {
      throw new IOException(t);
    }
  }
}
