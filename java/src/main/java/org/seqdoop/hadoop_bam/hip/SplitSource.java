// The bytes a FileVirtualSplit needs, read on demand for the streamed device decode
// (hbam_split_open_reader).  The reference's BAMRecordReader seeks an FSDataInputStream
// (BAMRecordReader.java:128-143 through util/WrapSeekable.java:42-87) and so reads only the blocks
// its split touches; this is the same for the device path: libhbam calls back (a Panama upcall
// stub bound to this object) with positioned reads of [offset, offset + len) for each window,
// from vStart's block to a bound past vEnd's block, every byte once.  Works for any Hadoop file
// system (HDFS, local, S3A): nothing maps, copies or page-locks the whole file.
package org.seqdoop.hadoop_bam.hip;

import java.io.IOException;
import java.lang.foreign.*;
import java.lang.invoke.MethodHandle;
import java.lang.invoke.MethodHandles;
import java.lang.invoke.MethodType;

import org.apache.hadoop.fs.FSDataInputStream;
import org.apache.hadoop.fs.FileSystem;
import org.apache.hadoop.fs.Path;

public final class SplitSource implements AutoCloseable {
  private static final MethodHandle READ;
  static {
    try {
      READ = MethodHandles.lookup().findVirtual(SplitSource.class, "read",
          MethodType.methodType(long.class, MemorySegment.class, long.class, long.class, MemorySegment.class));
    } catch (ReflectiveOperationException e) {
      throw new ExceptionInInitializerError(e);
    }
  }

  private final FSDataInputStream in;
  private final MemorySegment stub;  // hbam_read_fn
  private byte[] buf = new byte[1 << 22];
  private IOException failure;       // an upcall must not throw: kept and rethrown by the reader
  private long bytesRead;

  public SplitSource(FileSystem fs, Path file, Arena arena) throws IOException {
    in = fs.open(file);
    stub = Linker.nativeLinker().upcallStub(READ.bindTo(this),
        FunctionDescriptor.of(ValueLayout.JAVA_LONG, ValueLayout.ADDRESS, ValueLayout.JAVA_LONG,
                              ValueLayout.JAVA_LONG, ValueLayout.ADDRESS), arena);
  }

  /** hbam_read_fn: dst <- file bytes [off, off + len) (PositionedReadable.read); bytes read, or -1. */
  private long read(MemorySegment user, long off, long len, MemorySegment dst) {
    try {
      final MemorySegment d = dst.reinterpret(len);
      long done = 0;
      while (done < len) {
        final int k = in.read(off + done, buf, 0, (int) Math.min(buf.length, len - done));
        if (k <= 0) break;
        MemorySegment.copy(buf, 0, d, ValueLayout.JAVA_BYTE, done, k);
        done += k;
      }
      bytesRead += done;
      return done > 0 ? done : -1;
    } catch (IOException e) {
      failure = e;
      return -1;
    } catch (Throwable t) {
      failure = new IOException(t);
      return -1;
    }
  }

  /** hbam_split_open_reader over this file: the split's streamed decode (hbam_split_next). */
  public MemorySegment open(Hbam h, long fileLen, long vStart, long vEnd, int nRef, long windowBytes)
      throws IOException {
    final MemorySegment s;
    try {
      s = (MemorySegment) Hbam.SPLIT_OPEN_READER.invokeExact(h.context(), stub, MemorySegment.NULL, fileLen,
                                                             vStart, vEnd, nRef, windowBytes);
    } catch (Throwable t) {
      throw new IOException(t);
    }
    if (s.address() == 0) throw new IOException("hbam_split_open_reader: " + h.lastError());
    return s;
  }

  /** The read error behind a failed hbam_split_next, if any. */
  public IOException failure() { return failure; }

  public long bytesRead() { return bytesRead; }

  @Override public void close() throws IOException { in.close(); }
}
