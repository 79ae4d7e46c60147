// The device half of the Sort plugin (cli/plugins/Sort.java:84-205; SURVEY.md §8 a-13 and (e)):
// a node's decoded splits sorted on the GPU (hbam_sort_split: stable radix by the signed
// LongWritable key, the record bytes gathered in key order), cut at the TotalOrderPartitioner's
// split points (hbam_sort_partition: each partition's record and byte range, contiguous), and
// after the transport of the partitions the received concatenation sorted stably again
// (hbam_sort_received).  The transport between the GPUs of a node is libhbam's own RCCL
// exchange (Comm: hbam_comm_init, hbam_comm_split_points, hbam_sort_exchange — one rank per
// GPU, grouped ncclSend/ncclRecv over xGMI); a host with another transport (MPI, a Hadoop
// shuffle) uses partition() + received() around it instead.  Ties keep input order,
// so the output is ordered by (key, input, voffset): the documented tie-break.  Device buffers
// are hbam_device_alloc'ed and owned by the returned Run.
package org.seqdoop.hadoop_bam.hip;

import java.io.IOException;
import java.lang.foreign.*;

public final class HipSort {
  private static final ValueLayout.OfLong J = ValueLayout.JAVA_LONG;
  private static final AddressLayout A = ValueLayout.ADDRESS;

  /** hbam_sorted_run: n, payload_bytes, then the key / voffset / block_size / offsets / payload
   *  device arrays. */
  public static final StructLayout SORTED_RUN = MemoryLayout.structLayout(
      J.withName("n"), J.withName("payload_bytes"), A.withName("key"), A.withName("voffset"),
      A.withName("block_size"), A.withName("offsets"), A.withName("payload"));

  /** A sorted run in device memory (n records, their keys / voffsets / block sizes, payload
   *  offsets and packed SAMRecordWritable payloads). */
  public static final class Run implements AutoCloseable {
    public final MemorySegment struct;
    private final Hbam hbam;

    Run(Hbam h, MemorySegment s) { hbam = h; struct = s; }

    public long n() { return struct.get(J, 0); }
    public long payloadBytes() { return struct.get(J, 8); }
    public MemorySegment field(String f) {
      return struct.get(A, SORTED_RUN.byteOffset(MemoryLayout.PathElement.groupElement(f)));
    }

    @Override public void close() {
      for (String f : new String[] {"key", "voffset", "block_size", "offsets", "payload"}) free(hbam, field(f));
    }
  }

  private static MemorySegment alloc(Hbam h, long bytes) throws IOException {
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment out = a.allocate(A);
      final int rc = (int) Hbam.DEVICE_ALLOC.invokeExact(h.context(), Math.max(bytes, 1), out);
      if (rc != Hbam.OK) throw new IOException("hbam_device_alloc: " + h.lastError());
      return out.get(A, 0);
    } catch (IOException e) {
      throw e;
    } catch (Throwable t) {
      throw new IOException(t);
    }
  }

  private static void free(Hbam h, MemorySegment p) {
    try {
      final int rc = (int) Hbam.DEVICE_FREE.invokeExact(h.context(), p);
    } catch (Throwable t) {
      throw new RuntimeException(t);
    }
  }

  /** The size query, then the device buffers, then the call itself. */
  private interface RunCall { int call(MemorySegment run) throws Throwable; }

  private static Run run(Hbam h, RunCall c, Arena arena) throws IOException {
    final MemorySegment s = arena.allocate(SORTED_RUN);
    try {
      if (c.call(s) != Hbam.OK) throw new IOException("sorted-run size query: " + h.lastError());
      final long n = s.get(J, 0), nb = s.get(J, 8);
      s.set(A, 16, alloc(h, 8 * n));
      s.set(A, 24, alloc(h, 8 * n));
      s.set(A, 32, alloc(h, 4 * n));
      s.set(A, 40, alloc(h, 8 * (n + 1)));
      s.set(A, 48, alloc(h, nb));
      if (c.call(s) != Hbam.OK) throw new IOException("sorted run: " + h.lastError());
    } catch (IOException e) {
      throw e;
    } catch (Throwable t) {
      throw new IOException(t);
    }
    return new Run(h, s);
  }

  /** hbam_sort_split over a decoded split's device columns (Hbam.COLUMNS). */
  public static Run sortSplit(Hbam h, MemorySegment devColumns, Arena arena) throws IOException {
    return run(h, r -> (int) Hbam.SORT_SPLIT.invokeExact(h.context(), devColumns, r), arena);
  }

  /** TotalOrderPartitioner over a run: {recordBounds[], byteBounds[]} of the splitPoints.length+1
   *  partitions (partition k holds the keys in (splitPoints[k-1], splitPoints[k]]). */
  public static long[][] partition(Hbam h, Run run, long[] splitPoints) throws IOException {
    final int parts = splitPoints.length + 1;
    try (Arena a = Arena.ofConfined()) {
      final MemorySegment sp = a.allocateFrom(J, splitPoints.length == 0 ? new long[] {0} : splitPoints);
      final MemorySegment rb = a.allocate(J, parts + 1), bb = a.allocate(J, parts + 1);
      final int rc = (int) Hbam.SORT_PARTITION.invokeExact(h.context(), run.struct, sp, parts, rb, bb);
      if (rc != Hbam.OK) throw new IOException("hbam_sort_partition: " + h.lastError());
      return new long[][] {rb.toArray(J), bb.toArray(J)};
    } catch (IOException e) {
      throw e;
    } catch (Throwable t) {
      throw new IOException(t);
    }
  }

  /** One rank of the node's RCCL exchange (hbam_comm_*).  Rank 0 calls uniqueId(); the job ships
   *  the 128 bytes to every rank (e.g. a Configuration property, base64); every rank then
   *  constructs its Comm collectively on the context of its GPU. */
  public static final class Comm implements AutoCloseable {
    public static final int ID_BYTES = 128;
    private final Hbam hbam;
    private final MemorySegment comm;
    public final int nranks, rank;

    public static byte[] uniqueId() throws IOException {
      try (Arena a = Arena.ofConfined()) {
        final MemorySegment id = a.allocate(ID_BYTES);
        final int rc = (int) Hbam.COMM_UNIQUE_ID.invokeExact(id);
        if (rc != Hbam.OK) throw new IOException("hbam_comm_unique_id: RCCL unavailable (" + rc + ")");
        return id.toArray(ValueLayout.JAVA_BYTE);
      } catch (IOException e) {
        throw e;
      } catch (Throwable t) {
        throw new IOException(t);
      }
    }

    public Comm(Hbam h, byte[] uniqueId, int nranks, int rank) throws IOException {
      this.hbam = h;
      this.nranks = nranks;
      this.rank = rank;
      try (Arena a = Arena.ofConfined()) {
        final MemorySegment id = a.allocateFrom(ValueLayout.JAVA_BYTE, uniqueId);
        final MemorySegment out = a.allocate(A);
        final int rc = (int) Hbam.COMM_INIT.invokeExact(h.context(), id, nranks, rank, out);
        if (rc != Hbam.OK) throw new IOException("hbam_comm_init: " + h.lastError());
        comm = out.get(A, 0);
      } catch (IOException e) {
        throw e;
      } catch (Throwable t) {
        throw new IOException(t);
      }
    }

    /** The TotalOrderPartitioner's nranks-1 split points from every rank's sorted run (collective;
     *  the stand-in for InputSampler.writePartitionFile, Sort.java:154-157). */
    public long[] splitPoints(Run run, int samplesPerRank) throws IOException {
      try (Arena a = Arena.ofConfined()) {
        final MemorySegment sp = a.allocate(J, Math.max(nranks - 1, 1));
        final int rc = (int) Hbam.COMM_SPLIT_POINTS.invokeExact(hbam.context(), comm, run.struct, samplesPerRank, sp);
        if (rc != Hbam.OK) throw new IOException("hbam_comm_split_points: " + hbam.lastError());
        return java.util.Arrays.copyOf(sp.toArray(J), nranks - 1);
      } catch (IOException e) {
        throw e;
      } catch (Throwable t) {
        throw new IOException(t);
      }
    }

    /** This rank's slice of the total order: the partitions of every rank's run exchanged by key
     *  range and sorted again (collective). */
    public Run exchange(Run local, long[] splitPoints, Arena arena) throws IOException {
      final MemorySegment sp = arena.allocateFrom(J, splitPoints.length == 0 ? new long[] {0} : splitPoints);
      return run(hbam, r -> (int) Hbam.SORT_EXCHANGE.invokeExact(hbam.context(), comm, local.struct, sp, r), arena);
    }

    @Override public void close() {
      try { Hbam.COMM_DESTROY.invokeExact(comm); } catch (Throwable t) { throw new RuntimeException(t); }
    }
  }

  /** hbam_sort_received: the partitions a node received (concatenated in source order, device
   *  buffers) as one sorted run. */
  public static Run received(Hbam h, MemorySegment keys, MemorySegment voffsets, MemorySegment blockSizes,
                             MemorySegment payload, long n, Arena arena) throws IOException {
    return run(h, r -> (int) Hbam.SORT_RECEIVED.invokeExact(h.context(), keys, voffsets, blockSizes, payload, n, r),
               arena);
  }
}
