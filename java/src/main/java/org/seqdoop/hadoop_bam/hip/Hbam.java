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
      EEOF = -5, EREFID = -6, EDATA = -7, EMORE = -12, EINDEX = -13, ETRIBBLE = -14, ERUNTIME = -15,
      ENULL = -16, ECLASSCAST = -17;

  private static final Linker LINKER = Linker.nativeLinker();
  private static final SymbolLookup LIB = SymbolLookup.libraryLookup(
      Path.of(System.getProperty("hadoopbam.hip.lib", "libhbam.so")), Arena.global());

  private static MethodHandle fn(String name, FunctionDescriptor d) {
    return LINKER.downcallHandle(LIB.find(name).orElseThrow(), d);
  }

  private static final ValueLayout.OfLong J = ValueLayout.JAVA_LONG;
  private static final ValueLayout.OfInt I = ValueLayout.JAVA_INT;
  private static final AddressLayout A = ValueLayout.ADDRESS;

  static final MethodHandle CREATE = fn("hbam_create", FunctionDescriptor.of(A, I, A));
  static final MethodHandle DESTROY = fn("hbam_destroy", FunctionDescriptor.ofVoid(A));
  static final MethodHandle LAST_ERROR = fn("hbam_last_error", FunctionDescriptor.of(A, A));
  static final MethodHandle DECODE_SPLIT = fn("hbam_decode_split",
      FunctionDescriptor.of(I, A, A, I, J, J, J, J, J, I, A));
  static final MethodHandle COLUMNS_TO_HOST = fn("hbam_columns_to_host",
      FunctionDescriptor.of(I, A, A, A));
  static final MethodHandle FREE_HOST = fn("hbam_free_host_columns", FunctionDescriptor.ofVoid(A));
  // the drop-in reader's copy: key, voffset, rec_off, block_size + record bytes (context-owned, pinned)
  static final MethodHandle RECORDS_TO_HOST = fn("hbam_records_to_host",
      FunctionDescriptor.of(I, A, A, A));
  // the same into the split stream's own pinned staging (readers sharing a context stay apart)
  static final MethodHandle SPLIT_RECORDS_TO_HOST = fn("hbam_split_records_to_host",
      FunctionDescriptor.of(I, A, A, A));
  static final MethodHandle SPLIT_OPEN = fn("hbam_split_open",
      FunctionDescriptor.of(A, A, A, J, J, J, I, J));
  static final MethodHandle SPLIT_NEXT = fn("hbam_split_next", FunctionDescriptor.of(I, A, A));
  // split-local streamed read: positioned reads through an upcall stub (SplitSource)
  static final MethodHandle SPLIT_OPEN_READER = fn("hbam_split_open_reader",
      FunctionDescriptor.of(A, A, A, A, J, J, J, I, J));
  static final MethodHandle SPLIT_READ_BYTES = fn("hbam_split_read_bytes", FunctionDescriptor.of(J, A));
  static final MethodHandle HOST_REGISTER = fn("hbam_host_register", FunctionDescriptor.of(I, A, A, J));
  static final MethodHandle HOST_UNREGISTER = fn("hbam_host_unregister", FunctionDescriptor.of(I, A, A));
  static final MethodHandle SPLIT_CLOSE = fn("hbam_split_close", FunctionDescriptor.ofVoid(A));
  static final MethodHandle GUESS = fn("hbam_guess_bam_record_start",
      FunctionDescriptor.of(J, A, A, I, J, J, J, I, A));
  static final MethodHandle SPLITS = fn("hbam_probabilistic_splits",
      FunctionDescriptor.of(J, A, A, I, J, A, A, J, A, A));
  // split side over windows (a client never holds the file: HipBAMSplitGuesser,
  // HipBAMInputFormat, HipBGZFSplitGuesser)
  static final MethodHandle GUESS_WINDOW_LEN = fn("hbam_guess_window_len", FunctionDescriptor.of(J, J, J, J));
  static final MethodHandle GUESS_WINDOWS = fn("hbam_guess_windows",
      FunctionDescriptor.of(I, A, A, I, A, J, A, A, J, I, A, A));
  static final MethodHandle GUESS_BGZF_WINDOW_LEN = fn("hbam_guess_bgzf_window_len",
      FunctionDescriptor.of(J, J, J, J));
  static final MethodHandle GUESS_BGZF_WINDOW = fn("hbam_guess_bgzf_window",
      FunctionDescriptor.of(J, A, A, I, J, J, J, J, A));
  // Sort plugin path (HipSort, HipSortRecordReader)
  static final MethodHandle DEVICE_ALLOC = fn("hbam_device_alloc", FunctionDescriptor.of(I, A, J, A));
  static final MethodHandle DEVICE_FREE = fn("hbam_device_free", FunctionDescriptor.of(I, A, A));
  static final MethodHandle SORT_SPLIT = fn("hbam_sort_split", FunctionDescriptor.of(I, A, A, A));
  static final MethodHandle SORT_PARTITION = fn("hbam_sort_partition", FunctionDescriptor.of(I, A, A, A, I, A, A));
  static final MethodHandle SORT_RECEIVED = fn("hbam_sort_received", FunctionDescriptor.of(I, A, A, A, A, A, J, A));
  static final MethodHandle MERGE_REMAP = fn("hbam_merge_remap", FunctionDescriptor.of(I, A, A, A, I, A));
  static final MethodHandle REWRITE_GROUPS = fn("hbam_rewrite_groups", FunctionDescriptor.of(I, A, A, A, J, A, A));
  // the exchange over RCCL (HipSort.Comm): Sort.java:131-170's partitioner + shuffle
  static final MethodHandle COMM_UNIQUE_ID = fn("hbam_comm_unique_id", FunctionDescriptor.of(I, A));
  static final MethodHandle COMM_INIT = fn("hbam_comm_init", FunctionDescriptor.of(I, A, A, I, I, A));
  static final MethodHandle COMM_DESTROY = fn("hbam_comm_destroy", FunctionDescriptor.ofVoid(A));
  static final MethodHandle COMM_SPLIT_POINTS = fn("hbam_comm_split_points", FunctionDescriptor.of(I, A, A, A, I, A));
  static final MethodHandle SORT_EXCHANGE = fn("hbam_sort_exchange", FunctionDescriptor.of(I, A, A, A, A, A));
  static final MethodHandle SPLITS_WINDOWS = fn("hbam_probabilistic_splits_windows",
      FunctionDescriptor.of(J, A, A, J, A, I, A, J, A, A, J, A, A));
  // SURVEY.md §8 f-4: Summarize ranges, FixMate shuffle + reducer, device -> host copies
  static final MethodHandle SUMMARIZE = fn("hbam_summarize_ranges", FunctionDescriptor.of(I, A, A, A));
  static final MethodHandle NAME_ORDER = fn("hbam_name_order", FunctionDescriptor.of(I, A, A, A, J, A));
  static final MethodHandle FIXMATE = fn("hbam_fixmate", FunctionDescriptor.of(I, A, A, A, J, A));
  static final MethodHandle DOWNLOAD = fn("hbam_download", FunctionDescriptor.of(I, A, A, J, A));
  // SURVEY.md §8 f-3: BCF over BGZF (HipBCFSplitGuesser, HipBCFRecordReader)
  static final MethodHandle BCF_PARSE_HEADER = fn("hbam_bcf_parse_header", FunctionDescriptor.of(I, A, A, J, A));
  static final MethodHandle GUESS_BCF_WINDOW_LEN = fn("hbam_guess_bcf_window_len",
      FunctionDescriptor.of(J, J, J, J, I));
  static final MethodHandle GUESS_BCF_WINDOWS = fn("hbam_guess_bcf_windows",
      FunctionDescriptor.of(I, A, A, I, A, J, A, A, J, A, A, A));
  static final MethodHandle BCF_DECODE_SPLIT = fn("hbam_bcf_decode_split",
      FunctionDescriptor.of(I, A, A, I, J, J, J, A, J, J, A));

  /** hbam_bcf_header: n_contig, n_sample, n_dict, bgzf, header_len, first_voffset (32 bytes). */
  public static final StructLayout BCF_HEADER = MemoryLayout.structLayout(
      I.withName("n_contig"), I.withName("n_sample"), I.withName("n_dict"), I.withName("bgzf"),
      J.withName("header_len"), J.withName("first_voffset"));
  /** hbam_bcf_columns: counts/status, then rel, rec_off, data, data_len and the field arrays. */
  public static final StructLayout BCF_COLUMNS = MemoryLayout.structLayout(
      J.withName("n_records"), I.withName("status"), I.withName("pad0"), J.withName("err_record"),
      A.withName("rel"), A.withName("rec_off"), A.withName("data"), J.withName("data_len"), A.withName("key"),
      A.withName("l_shared"), A.withName("l_indiv"), A.withName("chrom"), A.withName("pos"), A.withName("rlen"),
      A.withName("qual"), A.withName("n_allele_info"), A.withName("n_fmt_sample"));

  /** hbam_ranges: n, status, pad, then the key / beg / end / rev / record device arrays. */
  public static final StructLayout RANGES = MemoryLayout.structLayout(
      J.withName("n"), I.withName("status"), I.withName("pad"), A.withName("key"), A.withName("beg"),
      A.withName("end"), A.withName("rev"), A.withName("record"));
  /** hbam_fixmate_run: n, payload_bytes, n_groups, status, pad, src / mate / offsets / payload. */
  public static final StructLayout FIXMATE_RUN = MemoryLayout.structLayout(
      J.withName("n"), J.withName("payload_bytes"), J.withName("n_groups"), I.withName("status"),
      I.withName("pad"), A.withName("src"), A.withName("mate"), A.withName("offsets"),
      A.withName("payload"));

  /** hbam_columns (include/hbam.h): 24 bytes of counts/status, then 27 pointer-sized slots
   *  (26 pointers and ubuf_len), 240 bytes in all. */
  public static final StructLayout COLUMNS = MemoryLayout.structLayout(
      J.withName("n_records"), I.withName("status"), I.withName("pad0"), J.withName("err_record"),
      A.withName("voffset"), A.withName("key"), A.withName("rec_off"), A.withName("ubuf"),
      J.withName("ubuf_len"), A.withName("block_size"), A.withName("ref_id"), A.withName("pos"),
      A.withName("l_read_name"), A.withName("mapq"), A.withName("bin"), A.withName("n_cigar"),
      A.withName("flag"), A.withName("l_seq"), A.withName("next_ref_id"), A.withName("next_pos"),
      A.withName("tlen"), A.withName("layout_ok"), A.withName("name_off"), A.withName("names"),
      A.withName("cigar_off"), A.withName("cigars"), A.withName("seq_off"), A.withName("seq"),
      A.withName("qual"), A.withName("aux_off"), A.withName("aux"));

  public static long offsetOf(String field) {
    return COLUMNS.byteOffset(MemoryLayout.PathElement.groupElement(field));
  }

  private final MemorySegment ctx;

  public Hbam(int device, boolean checkCrc) throws IOException {
    try (Arena a = Arena.ofConfined()) {
      MemorySegment opts = a.allocate(64);
      opts.set(I, 0, checkCrc ? 1 : 0);
      opts.set(I, 4, 1);  // validate_refs: BAMRecordCodec(header), BAMRecordReader.java:130
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
      case EIO: return new RuntimeIOException(new IOException(where));
      case EINDEX: return new IndexOutOfBoundsException(where);
      case ETRIBBLE: return new htsjdk.tribble.TribbleException(where);
      case ERUNTIME: return new RuntimeException("BCF2Codec.decode: " + where);
      case ENULL: return new NullPointerException(where);
      case ECLASSCAST: return new ClassCastException(where);
      default: return new RuntimeIOException("hbam error " + code + " at " + where);
    }
  }

  public String lastError() {
    try {
      MemorySegment s = (MemorySegment) LAST_ERROR.invokeExact(ctx);
      return s.reinterpret(4096).getString(0);
    } catch (Throwable t) {
      return "hbam_last_error failed: " + t;
    }
  }

  public MemorySegment context() { return ctx; }

  /** Bytes guessNextBAMRecordStart(beg, end) reads at beg (BAMSplitGuesser.java:114-125). */
  public static long guessWindowLen(long fileLen, long beg, long end) {
    try {
      return (long) GUESS_WINDOW_LEN.invokeExact(fileLen, beg, end);
    } catch (Throwable t) {
      throw new RuntimeException(t);
    }
  }

  /** Bytes guessNextBGZFBlockStart(beg, end) reads at beg (util/BGZFSplitGuesser.java:62-63). */
  public static long guessBgzfWindowLen(long fileLen, long beg, long end) {
    try {
      return (long) GUESS_BGZF_WINDOW_LEN.invokeExact(fileLen, beg, end);
    } catch (Throwable t) {
      throw new RuntimeException(t);
    }
  }

  /** Reads `len` bytes at `pos` the way BAMSplitGuesser buffers its window: read() calls until
   *  `len` bytes or end of stream (:116-125). */
  public static byte[] readWindow(htsjdk.samtools.seekablestream.SeekableStream in, long pos, int len)
      throws IOException {
    final byte[] b = new byte[len];
    in.seek(pos);
    int got = 0;
    while (got < len) {
      final int r = in.read(b, got, len - got);
      if (r < 0) break;
      got += r;
    }
    return got == len ? b : java.util.Arrays.copyOf(b, got);
  }

  /** hbam_guess_windows over k gathered windows (window i = windows[off[i], off[i+1])). */
  public void guessWindows(byte[] windows, long[] off, long fileLen, long[] beg, long[] end, int nRef,
                           long[] out, int[] err) throws IOException {
    final int k = beg.length;
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment w = a.allocate(Math.max(windows.length, 1));
      MemorySegment.copy(windows, 0, w, ValueLayout.JAVA_BYTE, 0, windows.length);
      final MemorySegment o = a.allocateFrom(J, off), b = a.allocateFrom(J, beg), e = a.allocateFrom(J, end);
      final MemorySegment r = a.allocate(J, Math.max(k, 1)), er = a.allocate(I, Math.max(k, 1));
      final int rc = (int) GUESS_WINDOWS.invokeExact(ctx, w, 0, o, fileLen, b, e, (long) k, nRef, r, er);
      if (rc != OK) throw new IOException("hbam_guess_windows: " + lastError());
      for (int i = 0; i < k; ++i) {
        out[i] = r.getAtIndex(J, i);
        err[i] = er.getAtIndex(I, i);
      }
    } catch (IOException | RuntimeException ex) {
      throw ex;
    } catch (Throwable t) {
      throw new IOException(t);
    }
  }

  /** hbam_download: `bytes` of library-owned device memory into a new host segment of `arena`. */
  public MemorySegment download(MemorySegment dev, long bytes, Arena arena) {
    final MemorySegment h = arena.allocate(Math.max(bytes, 1), 16);
    try {
      final int rc = (int) DOWNLOAD.invokeExact(ctx, dev, bytes, h);
      if (rc != OK) throw exceptionFor(rc, "hbam_download: " + lastError());
    } catch (RuntimeException e) {
      throw e;
    } catch (Throwable t) {
      throw new RuntimeException(t);
    }
    return h;
  }

  @Override public void close() {
    try { DESTROY.invokeExact(ctx); } catch (Throwable t) { throw new RuntimeException(t); }
  }
}
