// Panama FFI (JDK 22+) binding of libhbam.so (include/hbam.h) — the shim a maintainer adds
// under Hadoop-BAM so BAMRecordReader / BAMInputFormat / BAMSplitGuesser keep their API and
// run the MI355X path.  Compiles with any JDK >= 22 (none in the build image: source only).
package org.seqdoop.hadoop_bam.hip;

import java.io.IOException;
import java.lang.foreign.*;
import java.lang.invoke.MethodHandle;
import java.nio.file.Path;

import htsjdk.samtools.FileTruncatedException;
import htsjdk.samtools.SAMFormatException;
import htsjdk.samtools.util.RuntimeEOFException;
import htsjdk.samtools.util.RuntimeIOException;

public final class Hbam implements AutoCloseable {
  public static final int OK = 0, EIO = -1, ETRUNC = -2, EFORMAT = -3, ERUNTIMEIO = -4,
      EEOF = -5, EREFID = -6, EDATA = -7;

  private static final Linker LINKER = Linker.nativeLinker();
  private static final SymbolLookup LIB = SymbolLookup.libraryLookup(
      Path.of(System.getProperty("hadoopbam.hip.lib", "libhbam.so")), Arena.global());

  private static MethodHandle fn(String name, FunctionDescriptor d) {
    return LINKER.downcallHandle(LIB.find(name).orElseThrow(), d);
  }

  static final MethodHandle CREATE = fn("hbam_create",
      FunctionDescriptor.of(ValueLayout.ADDRESS, ValueLayout.JAVA_INT, ValueLayout.ADDRESS));
  static final MethodHandle DESTROY = fn("hbam_destroy",
      FunctionDescriptor.ofVoid(ValueLayout.ADDRESS));
  static final MethodHandle DECODE_SPLIT = fn("hbam_decode_split",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.ADDRESS,
          ValueLayout.JAVA_INT, ValueLayout.JAVA_LONG, ValueLayout.JAVA_LONG,
          ValueLayout.JAVA_LONG, ValueLayout.JAVA_LONG, ValueLayout.JAVA_LONG,
          ValueLayout.JAVA_INT, ValueLayout.ADDRESS));
  static final MethodHandle COLUMNS_TO_HOST = fn("hbam_columns_to_host",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.ADDRESS,
          ValueLayout.ADDRESS));
  static final MethodHandle FREE_HOST = fn("hbam_free_host_columns",
      FunctionDescriptor.ofVoid(ValueLayout.ADDRESS));
  static final MethodHandle GUESS = fn("hbam_guess_bam_record_start",
      FunctionDescriptor.of(ValueLayout.JAVA_LONG, ValueLayout.ADDRESS, ValueLayout.ADDRESS,
          ValueLayout.JAVA_INT, ValueLayout.JAVA_LONG, ValueLayout.JAVA_LONG,
          ValueLayout.JAVA_LONG, ValueLayout.JAVA_INT, ValueLayout.ADDRESS));
  static final MethodHandle SPLITS = fn("hbam_probabilistic_splits",
      FunctionDescriptor.of(ValueLayout.JAVA_LONG, ValueLayout.ADDRESS, ValueLayout.ADDRESS,
          ValueLayout.JAVA_INT, ValueLayout.JAVA_LONG, ValueLayout.ADDRESS, ValueLayout.ADDRESS,
          ValueLayout.JAVA_LONG, ValueLayout.ADDRESS, ValueLayout.ADDRESS));

  /** hbam_columns (include/hbam.h): 8-byte fields, pointers as addresses. */
  public static final MemoryLayout COLUMNS = MemoryLayout.structLayout(
      ValueLayout.JAVA_LONG.withName("n_records"), ValueLayout.JAVA_INT.withName("status"),
      ValueLayout.JAVA_INT.withName("pad0"), ValueLayout.JAVA_LONG.withName("err_record"),
      MemoryLayout.sequenceLayout(28, ValueLayout.ADDRESS).withName("ptrs_and_len"));

  private final MemorySegment ctx;

  public Hbam(int device, boolean checkCrc) throws IOException {
    try (Arena a = Arena.ofConfined()) {
      MemorySegment opts = a.allocate(64);
      opts.set(ValueLayout.JAVA_INT, 0, checkCrc ? 1 : 0);
      opts.set(ValueLayout.JAVA_INT, 4, 1);  // validate_refs: BAMRecordCodec(header)
      ctx = (MemorySegment) CREATE.invokeExact(device, opts);
    } catch (Throwable t) {
      throw new IOException(t);
    }
    if (ctx.address() == 0) throw new IOException("no HIP device " + device);
  }

  /** Maps an hbam status to the exception the reference raises at that point. */
  public static RuntimeException exceptionFor(int code, String where) {
    switch (code) {
      case ETRUNC: return new FileTruncatedException(where);
      case EFORMAT: return new SAMFormatException(where);
      case ERUNTIMEIO: return new RuntimeIOException(where);
      case EEOF: return new RuntimeEOFException(where);
      case EREFID: return new IllegalArgumentException(where);
      case EDATA: return new RuntimeException(new java.util.zip.DataFormatException(where));
      default: return new RuntimeIOException("hbam error " + code + " at " + where);
    }
  }

  public MemorySegment context() { return ctx; }

  @Override public void close() {
    try { DESTROY.invokeExact(ctx); } catch (Throwable t) { throw new RuntimeException(t); }
  }
}
