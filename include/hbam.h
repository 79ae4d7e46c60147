/* hbam.h — C ABI of the MI355X-native BAM read path (libhbam.so).
 *
 * Drop-in boundary for Hadoop-BAM's BAM input path.  The reference's Java classes
 * (org.seqdoop.hadoop_bam.*) keep their API and bind these entry points through
 * Panama FFI / JNI.  Every entry point names the reference
 * interface it replaces.  Plain C: pointers + sizes, no C++ or torch types, no
 * exceptions across the boundary.  Negative return codes map 1:1 onto the Java
 * exception the reference raises at the same point:
 *
 *   HBAM_EIO          java.io.IOException
 *   HBAM_ETRUNC       htsjdk.samtools.FileTruncatedException
 *   HBAM_EFORMAT      htsjdk.samtools.SAMFormatException
 *   HBAM_ERUNTIMEIO   htsjdk.samtools.util.RuntimeIOException
 *   HBAM_EEOF         htsjdk.samtools.util.RuntimeEOFException
 *   HBAM_EREFID       IllegalArgumentException (reference index not in dictionary)
 *   HBAM_EDATA        RuntimeException(java.util.zip.DataFormatException)
 *   HBAM_EINDEX       IndexOutOfBoundsException
 *   HBAM_ETRIBBLE     htsjdk TribbleException (BCF)
 *   HBAM_ERUNTIME     another RuntimeException out of BCF2Codec.decode (BCF, unpinned)
 *   HBAM_ENULL        NullPointerException (multi-input Sort's group rewrite, cli/Utils.java:316-323)
 *   HBAM_ECLASSCAST   ClassCastException (an RG / PG attribute that is not a string)
 *
 * Library-specific codes (no reference counterpart): HBAM_ENOMEM, HBAM_EUNSUPPORTED
 * (BGZF block with ISIZE > 65536), HBAM_EDEVICE (HIP error), HBAM_EINVAL, HBAM_EMORE
 * (the compressed window handed in ends before the split's last record).
 *
 * Inputs: an argument with `on_device` = 0 is host memory, copied in by the call; with
 * `on_device` = 1 it is a device pointer read in place, and the kernels read whole 16-byte
 * quads and fixed-size windows past the last byte, so 64 readable bytes must follow `len`
 * (their contents do not matter).  Host inputs get that padding from the library.
 *
 * Threading: a context owns one HIP stream and is single-threaded; separate contexts
 * (one per Hadoop task thread) are independent.  Device buffers returned in
 * hbam_columns are owned by the context and stay valid until the next decode call on
 * that context or hbam_release_columns().
 */
#ifndef HBAM_H
#define HBAM_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HBAM_OK 0
#define HBAM_EIO (-1)
#define HBAM_ETRUNC (-2)
#define HBAM_EFORMAT (-3)
#define HBAM_ERUNTIMEIO (-4)
#define HBAM_EEOF (-5)
#define HBAM_EREFID (-6)
#define HBAM_EDATA (-7)
#define HBAM_ENOMEM (-8)
#define HBAM_EUNSUPPORTED (-9)
#define HBAM_EDEVICE (-10)
#define HBAM_EINVAL (-11)
#define HBAM_EMORE (-12)
#define HBAM_EINDEX (-13) /* IndexOutOfBoundsException (Summarize.java:715 on a record without a range) */
#define HBAM_ETRIBBLE (-14) /* htsjdk TribbleException (BCF2Codec: unreadable / inconsistent BCF record) */
#define HBAM_ERUNTIME (-15) /* another RuntimeException escaping BCF2Codec.decode (restated, unpinned) */
#define HBAM_ENULL (-16) /* NullPointerException (cli/Utils.java:316-323: a group lookup without a table) */
#define HBAM_ECLASSCAST (-17) /* ClassCastException ((String) of a non-string RG / PG attribute) */

typedef struct hbam_ctx hbam_ctx;

/* Configuration knobs (Hadoop Configuration properties in the Java shim):
 *   check_crc      hadoopbam.hip.check-crc: BlockCompressedInputStream.setCheckCrcs
 *                  (off in BAMRecordReader, on in the split guessers)
 *   validate_refs  1 = BAMRecordCodec(header) as BAMRecordReader.java:130 builds it
 *                  (refID / mate refID must lie in [-1, n_ref)); 0 = LazyBAMRecordFactory */
typedef struct hbam_opts {
  int32_t check_crc;
  int32_t validate_refs;
  int32_t reserved[14];  /* must be zero */
} hbam_opts;

typedef struct hbam_header {
  int32_t l_text;
  int32_t n_ref;           /* SAMFileHeader.getSequenceDictionary().size() */
  uint64_t header_ulen;    /* uncompressed bytes of the BAM header */
  uint64_t first_voffset;  /* virtual offset of the first record */
} hbam_header;

typedef struct hbam_block {
  uint64_t coff;   /* file offset of the BGZF block */
  uint32_t clen;   /* BSIZE + 1 */
  uint32_t isize;  /* ISIZE footer */
  uint32_t crc;    /* CRC32 footer */
  uint32_t pad;
} hbam_block;

/* Decoded split, struct-of-arrays.  In hbam_decode_split's output every pointer is a
 * device pointer owned by the context; after hbam_columns_to_host they are host
 * pointers owned by the caller (free with hbam_free_host_columns).  In the host copy, ubuf
 * holds exactly the records' bytes (each record's block_size field + record, i.e. the
 * SAMRecordWritable wire form) and rec_off is relative to it. */
typedef struct hbam_columns {
  uint64_t n_records;
  int32_t status;       /* HBAM_OK, or the exception nextKeyValue()/initialize() raises */
  int32_t pad0;
  uint64_t err_record;  /* record index at which `status` is raised */
  uint64_t* voffset;    /* bci.getFilePointer() before each record */
  int64_t* key;         /* BAMRecordReader.getKey(record) (LongWritable key) */
  uint64_t* rec_off;    /* offset of each record's block_size field in ubuf */
  uint8_t* ubuf;        /* inflated stream of the split (SAMRecordWritable payloads) */
  uint64_t ubuf_len;
  int32_t* block_size;
  int32_t* ref_id;
  int32_t* pos;         /* 0-based */
  uint8_t* l_read_name;
  uint8_t* mapq;
  uint16_t* bin;
  uint16_t* n_cigar;
  uint16_t* flag;
  int32_t* l_seq;
  int32_t* next_ref_id;
  int32_t* next_pos;
  int32_t* tlen;
  uint8_t* layout_ok;   /* 0: variable block inconsistent with the fixed lengths */
  uint64_t* name_off;   /* n+1 offsets into names (l_read_name bytes each, incl. NUL) */
  uint8_t* names;
  uint64_t* cigar_off;  /* n+1 offsets (in u32 ops) into cigars */
  uint32_t* cigars;
  uint64_t* seq_off;    /* n+1 offsets into seq (unpacked "=ACMGRSVTWYHKDBN") and qual */
  uint8_t* seq;
  uint8_t* qual;
  uint64_t* aux_off;    /* n+1 offsets into aux (raw typed tags) */
  uint8_t* aux;
} hbam_columns;

/* Per-stage device times of the last call, milliseconds (HIP events on the context's
 * stream), for the roofline report. */
typedef struct hbam_timing {
  double scan_ms, inflate_ms, crc_ms, walk_ms, decode_ms, pools_ms, total_ms;
  double huffman_ms, resolve_ms; /* inflate = Huffman pass (k_inflate_tokens) + k_resolve (LZ77) */
  uint64_t n_blocks, comp_bytes, ubuf_bytes, n_records, pool_bytes;
  double exchange_ms; /* hbam_sort_exchange: the grouped ncclSend/ncclRecv on the context stream */
} hbam_timing;

/* ---- context ---------------------------------------------------------------------- */
hbam_ctx* hbam_create(int device_ordinal, const hbam_opts* opts);
void hbam_destroy(hbam_ctx* ctx);
const char* hbam_last_error(const hbam_ctx* ctx);
void* hbam_stream(hbam_ctx* ctx); /* hipStream_t of the context */
int hbam_get_timing(const hbam_ctx* ctx, hbam_timing* out);

/* ---- device staging (the Java shim maps HDFS bytes into pinned buffers) ---------- */
int hbam_upload(hbam_ctx* ctx, const uint8_t* host, uint64_t len, uint8_t** dev_out);
int hbam_device_free(hbam_ctx* ctx, uint8_t* dev);
/* page-lock / release a caller-owned host range (hipHostRegister) so hbam_split_next's window
 * copies run asynchronously beside the decode; memory pinned by another HIP runtime in the
 * process (PyTorch-ROCm's) is pageable to this library */
int hbam_host_register(hbam_ctx* ctx, void* host, uint64_t len);
int hbam_host_unregister(hbam_ctx* ctx, void* host);
/* copy `bytes` of library-owned device memory (e.g. an f-4 output) to host memory, ordered after
 * the context's work */
int hbam_download(hbam_ctx* ctx, const void* dev, uint64_t bytes, void* host);

/* ---- SAMHeaderReader.readSAMHeaderFrom (util/SAMHeaderReader.java:53-72) ----------
 * `file` holds the start of the BAM file (host or device per `on_device`). */
int hbam_parse_header(hbam_ctx* ctx, const uint8_t* file, int on_device, uint64_t len,
                      hbam_header* out);

/* ---- BGZF block table: [htsjdk] BlockCompressedInputStream.readBlock framing;
 * util/BGZFBlockIndexer.java:130-181 (skipBlock).  Chain from offset 0 of `comp`. */
int hbam_scan_blocks(hbam_ctx* ctx, const uint8_t* comp, int on_device, uint64_t len,
                     uint64_t base_off, hbam_block* out, uint64_t cap, uint64_t* n_out);

/* ---- batched inflate: [htsjdk] BlockGunzipper.unzipBlock (JDK zlib).  Blocks are
 * relative to `comp`; output concatenated into host `out` at out_off (n+1 entries,
 * exclusive scan of ISIZE, filled by the call).  blk_status: 0, HBAM_EFORMAT (short
 * output / CRC mismatch), HBAM_EDATA (DataFormatException). */
int hbam_inflate(hbam_ctx* ctx, const uint8_t* comp, int on_device, uint64_t comp_len,
                 const hbam_block* blks, uint64_t n, int check_crc, uint8_t* out,
                 uint64_t out_cap, uint64_t* out_off, int32_t* blk_status);

/* ---- BAMRecordReader.initialize + nextKeyValue loop (BAMRecordReader.java:108-188)
 * over FileVirtualSplit [v_start, v_end) (FileVirtualSplit.java:38-92).
 * `comp` = bytes [comp_base, comp_base+comp_len) of a file of length file_len (a window).
 * n_ref < 0: parse it from the header (comp must then start at file offset 0).
 * Windows: when the window ends before the split does, out->status = HBAM_EMORE, the first
 * n_records records are final, and voffset[n_records] (device) is the virtual offset to
 * resume from (v_start when n_records == 0 and no column was produced: the window is too
 * small); the next window must start at or before that offset's BGZF block.  Resuming at
 * that offset gives exactly the records (and the exception) one whole-file call gives. */
int hbam_decode_split(hbam_ctx* ctx, const uint8_t* comp, int on_device, uint64_t comp_base,
                      uint64_t comp_len, uint64_t file_len, uint64_t v_start, uint64_t v_end,
                      int32_t n_ref, hbam_columns* out);
int hbam_columns_to_host(hbam_ctx* ctx, const hbam_columns* dev, hbam_columns* host);
/* Records-only host copy for the drop-in reader: BAMRecordReader.nextKeyValue
 * (BAMRecordReader.java:172-188) hands out one record at a time and needs only its bytes, its key
 * and (getProgress, :157-168) its virtual offset.  host gets n_records, status, err_record, key,
 * voffset, block_size, rec_off (relative to host->ubuf) and ubuf = exactly the records' bytes
 * (each record's block_size field + record); every other pointer is NULL.  The arrays live in
 * pinned host memory owned by the context, valid until the next hbam_records_to_host or
 * hbam_destroy on it (never pass them to hbam_free_host_columns): one consumer per context — a
 * reader among several on one context takes hbam_split_records_to_host instead.  Copies 28 B per
 * record plus the record bytes (columns_to_host copies every pool too: about twice as much).
 * Precondition: `dev` holds a decoded split's columns (hbam_decode_split, hbam_split_next,
 * hbam_rewrite_groups), whose records lie back to back in ubuf in index order; columns whose
 * records are permuted or not contiguous return HBAM_EINVAL. */
int hbam_records_to_host(hbam_ctx* ctx, const hbam_columns* dev, hbam_columns* host);
/* Streamed split read: BAMRecordReader over FileVirtualSplit
 * [v_start, v_end) of a file the caller holds in host memory (e.g. mmap; only the split's
 * windows are copied, see hbam_split_open_reader for the bound), decoded in windows
 * of about window_bytes compressed bytes.  While window k decodes, the predicted window k+1
 * is copied to the device on a second HIP stream.  hbam_split_next fills `out` (device
 * columns, valid until the next call on the stream's context) with the next window's
 * records and returns 1, returns 0 once the split is exhausted, <0 on a library error;
 * out->status != HBAM_OK (never HBAM_EMORE) is the exception nextKeyValue raises after
 * out->n_records records, and ends the stream. */
typedef struct hbam_split_stream hbam_split_stream;
hbam_split_stream* hbam_split_open(hbam_ctx* ctx, const uint8_t* file, uint64_t file_len,
                              uint64_t v_start, uint64_t v_end, int32_t n_ref,
                              uint64_t window_bytes);
/* Split-local streamed read (BAMRecordReader.java:128-143 reads only the blocks the split touches,
 * through FSDataInputStream.seek, util/WrapSeekable.java:42-87): the caller's read(user, offset,
 * len, dst) fills dst with file bytes [offset, offset + len) and returns the bytes read (> 0; a
 * positioned read such as FSDataInputStream.read(long, byte[], int, int) or pread).  Only bytes
 * from v_start's block to a bound past v_end's block are read (at most (v_end >> 16) + 192 KiB
 * unless a record runs longer), each at most once: the windows' overlap is re-used from the
 * previous window's pinned staging.  Same output as hbam_split_open on the whole file.
 * hbam_split_read_bytes: the bytes requested from `read` so far. */
typedef int64_t (*hbam_read_fn)(void* user, uint64_t offset, uint64_t len, uint8_t* dst);
hbam_split_stream* hbam_split_open_reader(hbam_ctx* ctx, hbam_read_fn read, void* user, uint64_t file_len,
                                     uint64_t v_start, uint64_t v_end, int32_t n_ref,
                                     uint64_t window_bytes);
int hbam_split_next(hbam_split_stream* s, hbam_columns* out);
/* bytes copied host->device and the copies' wall time (ms) so far */
int hbam_split_stats(const hbam_split_stream* s, uint64_t* h2d_bytes, double* h2d_ms, uint64_t* windows);
uint64_t hbam_split_read_bytes(const hbam_split_stream* s);
void hbam_split_close(hbam_split_stream* s);
/* hbam_records_to_host into the split stream's own pinned staging: valid until the next call on
 * this stream or hbam_split_close, whatever other streams of the same context do (the drop-in
 * readers: several BAMRecordReaders may share one context). */
int hbam_split_records_to_host(hbam_split_stream* s, const hbam_columns* dev, hbam_columns* host);
void hbam_free_host_columns(hbam_columns* host);
void hbam_release_columns(hbam_ctx* ctx, hbam_columns* dev);

/* ---- BAMSplitGuesser.guessNextBAMRecordStart (BAMSplitGuesser.java:109-212) -------
 * Returns the virtual offset of the guessed record, or `end`.  `file` is the whole file
 * (host or device).  *err = exception escaping the guesser (HBAM_OK normally). */
int64_t hbam_guess_bam_record_start(hbam_ctx* ctx, const uint8_t* file, int on_device,
                                    uint64_t file_len, int64_t beg, int64_t end, int32_t n_ref,
                                    int32_t* err);
/* batched guesses: k independent [beg[i], end[i]) ranges (one guesser per range). */
int hbam_guess_batch(hbam_ctx* ctx, const uint8_t* file, int on_device, uint64_t file_len,
                     const int64_t* beg, const int64_t* end, uint64_t k, int32_t n_ref,
                     int64_t* out, int32_t* err);

/* Windowed guesses: the bytes guessNextBAMRecordStart reads are the window
 * file[beg, beg + min((int)(end-beg), 262139)) cut at the end of the file
 * (BAMSplitGuesser.java:114-125; hbam_guess_window_len gives its length), so a client that
 * does not hold the file (a JVM computing getSplits over HDFS) gathers those k windows and
 * passes them concatenated: window i = windows[win_off[i], win_off[i+1]) (win_off: host,
 * k+1 entries, win_off[0] = 0; a length other than hbam_guess_window_len -> HBAM_EINVAL).
 * Same results as hbam_guess_batch over the whole file.  hbam_guess_batch itself stages only
 * these windows when `file` is on the host. */
uint64_t hbam_guess_window_len(uint64_t file_len, int64_t beg, int64_t end);
int hbam_guess_windows(hbam_ctx* ctx, const uint8_t* windows, int on_device, const uint64_t* win_off,
                       uint64_t file_len, const int64_t* beg, const int64_t* end, uint64_t k,
                       int32_t n_ref, int64_t* out, int32_t* err);

/* ---- BGZFSplitGuesser.guessNextBGZFBlockStart (util/BGZFSplitGuesser.java:51-92) ---
 * The guesser reads one window of min((int)(end-beg), 131069) bytes at beg (:62-63):
 * hbam_guess_bgzf_window takes that window alone (wlen = hbam_guess_bgzf_window_len). */
int64_t hbam_guess_bgzf_block_start(hbam_ctx* ctx, const uint8_t* file, int on_device,
                                    uint64_t file_len, int64_t beg, int64_t end, int32_t* err);
uint64_t hbam_guess_bgzf_window_len(uint64_t file_len, int64_t beg, int64_t end);
int64_t hbam_guess_bgzf_window(hbam_ctx* ctx, const uint8_t* window, int on_device, uint64_t wlen,
                               uint64_t file_len, int64_t beg, int64_t end, int32_t* err);

/* ---- BAMInputFormat.getSplits for one file (BAMInputFormat.java:76-103,163-224):
 * Hadoop FileSplits [beg[i], end[i]) -> FileVirtualSplits.  Returns the number of
 * virtual splits, or a negative code ("no reads in first split" -> HBAM_EIO).
 * hbam_probabilistic_splits_windows: the same from the file's first head_len bytes (host; the
 * BAM header — HBAM_ETRUNC: too short, read more) and the guess windows of the n FileSplits
 * (as hbam_guess_windows), for a client that reads only those bytes. */
int64_t hbam_probabilistic_splits(hbam_ctx* ctx, const uint8_t* file, int on_device,
                                  uint64_t file_len, const uint64_t* beg, const uint64_t* end,
                                  uint64_t n, uint64_t* v_start, uint64_t* v_end);
int64_t hbam_probabilistic_splits_windows(hbam_ctx* ctx, const uint8_t* head, uint64_t head_len,
                                          const uint8_t* windows, int on_device, const uint64_t* win_off,
                                          uint64_t file_len, const uint64_t* beg, const uint64_t* end,
                                          uint64_t n, uint64_t* v_start, uint64_t* v_end);

/* ---- Sort plugin path (Sort.java:84-188, SortReducer 191-205) ------
 * hbam_sort_keys: stable sort of n LongWritable keys (signed i64, Hadoop's comparator) on
 * the device; replaces the MapReduce shuffle sort of Sort's map output.  Ties keep input
 * order, so over one split's decode (voffset order) the result is ordered by (key, voffset).
 * keys (device, i64[n]) is not modified; perm (device, u32[n]) receives the source index of
 * each output position; keys_out (device, i64[n], may be NULL) the sorted keys.  n < 2^32.
 * Timing: total_ms = device time, n_blocks = radix passes run. */
int hbam_sort_keys(hbam_ctx* ctx, const int64_t* keys, uint64_t n, int64_t* keys_out,
                   uint32_t* perm);
/* hbam_gather_records: SAMRecordWritable.write (block_size + record bytes, SAMRecordWritable
 * .java:62-63) of records perm[0..n) (perm NULL = identity) from an inflated stream (ubuf,
 * rec_off, block_size: a decoded split's columns, or a received exchange buffer) into out,
 * packed; out_off (device, u64[n+1]) gets the exclusive scan of lengths.  out == NULL: size
 * query (total_bytes only).  All pointers device pointers except total_bytes (host). */
int hbam_gather_records(hbam_ctx* ctx, const uint8_t* ubuf, const uint64_t* rec_off,
                        const int32_t* block_size, const uint32_t* perm, uint64_t n, uint8_t* out,
                        uint64_t out_cap, uint64_t* out_off, uint64_t* total_bytes);
/* ---- Sort plugin, one rank's steps (Sort.java:131-170, SortRecordReader :279-295) ----------
 * A sorted run: records in (key, input order) order with their voffsets, block sizes and packed
 * SAMRecordWritable payloads (block_size field + record, SAMRecordWritable.java:62-63).  All
 * pointers are caller-owned device buffers (hbam_device_alloc): call with payload == NULL
 * first to get n and payload_bytes, then with key[n], voffset[n], block_size[n],
 * offsets[n+1] (payload offsets) and payload[payload_bytes].  A Java host drives the plugin as
 *   decode (hbam_decode_split) -> hbam_sort_split -> hbam_sort_partition with the
 *   TotalOrderPartitioner split points -> its own transport of each partition's slice ->
 *   hbam_sort_received on the concatenation of what it received (in source order).
 * Ties keep input order, so a run is ordered by (key, file order): the documented tie-break. */
typedef struct hbam_sorted_run {
  uint64_t n;
  uint64_t payload_bytes;
  int64_t* key;
  int64_t* voffset;
  int32_t* block_size;
  uint64_t* offsets;
  uint8_t* payload;
} hbam_sorted_run;
/* device buffer of `bytes` bytes followed by 64 more readable bytes, so it may be passed back as a
 * device-resident input (the 64-byte rule above); free with hbam_device_free */
int hbam_device_alloc(hbam_ctx* ctx, uint64_t bytes, void** dev_out);
/* the records of a decoded split (device columns) as a sorted run */
int hbam_sort_split(hbam_ctx* ctx, const hbam_columns* dv, hbam_sorted_run* out);
/* TotalOrderPartitioner (Sort.java:149) over a sorted run: partition k (0 <= k < nparts) holds
 * the keys in (split_points[k-1], split_points[k]] (host array of nparts-1 signed keys);
 * rec_bounds / byte_bounds (host, nparts+1) get each partition's record and payload ranges. */
int hbam_sort_partition(hbam_ctx* ctx, const hbam_sorted_run* run, const int64_t* split_points,
                        uint32_t nparts, uint64_t* rec_bounds, uint64_t* byte_bounds);
/* Multi-input Sort (Sort.java:111-113 + SortRecordReader.nextKeyValue :279-295): when the inputs'
 * sequence dictionaries differ, Utils.correctSAMRecordForMerging (cli/Utils.java:286-313) maps
 * every record of input i onto the merged dictionary.  hbam_merge_remap does it on the device
 * over a decoded split (dv, modified in place): refID -> ref_map[refID] (host, n_in entries =
 * the input's dictionary size; -1 stays -1), next refID likewise for paired reads (flag 0x1),
 * in the columns and in the record bytes, and the key recomputed (BAMRecordReader.getKey) where
 * refID changed.  *bad_record = the first record whose new index lies outside its own input's
 * dictionary (htsjdk resolves setReferenceIndex against the record's header: the reference
 * throws IllegalArgumentException there), else UINT64_MAX.  Run it before hbam_sort_split. */
int hbam_merge_remap(hbam_ctx* ctx, hbam_columns* dv, const int32_t* ref_map, int32_t n_in,
                     uint64_t* bad_record);
/* Multi-input Sort, continued: Utils.correctSAMRecordForMerging's program-group / read-group
 * rewrite (cli/Utils.java:314-324) when SamFileHeaderMerger reports ID collisions.  Over a decoded
 * split of input h (dv, after hbam_merge_remap): every record carrying the tag gets
 * setAttribute(tag, getProgramGroupId(h, value)) — for RG too (the reference's quirk: RG values are
 * looked up in the PROGRAM-group table) — and is re-encoded as BAMRecordCodec.encode writes a record
 * whose attributes changed (integer tags re-typed, odd sequence pad nibble zeroed, absent qualities
 * 0xFF, bin 0 when unplaced; restated from htsjdk 1.131, parity unpinned).  `table` (host) holds, for
 * PG then RG: u8 mode (0 no collisions of that kind: untouched; 1 translate; 2 h has no @PG record:
 * NullPointerException at the first record carrying the tag), u16 count, then `count` entries
 * {u16 old_len, old bytes, i16 new_len (-1: the value is not in the table -> tag removed; not needed:
 * an absent value is removed too), new bytes}.  On return dv's ubuf / ubuf_len / rec_off / block_size
 * point at the rewritten records (context-owned; the aux pool is not refreshed) and *status is HBAM_OK,
 * or the exception raised at record *err_record (HBAM_ENULL, HBAM_ECLASSCAST, HBAM_EFORMAT): dv then
 * holds the records before it. */
int hbam_rewrite_groups(hbam_ctx* ctx, hbam_columns* dv, const uint8_t* table, uint64_t table_len,
                        int32_t* status, uint64_t* err_record);
/* receive side: n records (device key/voffset/block_size and their packed payload, chunks in
 * source-rank order) as a sorted run */
int hbam_sort_received(hbam_ctx* ctx, const int64_t* key, const int64_t* voffset,
                       const int32_t* block_size, const uint8_t* payload, uint64_t n,
                       hbam_sorted_run* out);

/* ---- Sort plugin exchange over RCCL (Sort.java:131-170: the TotalOrderPartitioner + Hadoop
 * shuffle between map and reduce tasks; SURVEY.md §8(b) hbam_sort_multi_gpu, §8(e) steps 2-3).
 * One rank per GPU.  RCCL (librccl.so.1) is loaded on the first hbam_comm_init.
 *   rank 0: hbam_comm_unique_id(id); the job ships the 128 bytes to every rank (a Hadoop
 *           Configuration property, MPI, torch.distributed.broadcast);
 *   every rank, collectively: hbam_comm_init(ctx, id, nranks, rank, &comm);
 *   every rank, collectively: hbam_comm_split_points(ctx, comm, run, samples, sp) — regular
 *           samples of each rank's sorted keys all-gathered (ncclAllGather), the nranks-1 split
 *           points their quantiles (deterministic; the reference's RandomSampler is unseeded);
 *   every rank, collectively, twice: hbam_sort_exchange(ctx, comm, run, sp, out) — first with
 *           out->payload == NULL: the partition of `run` (hbam_sort_partition) and the count
 *           all-gather, out->n / out->payload_bytes = what this rank will receive; then with
 *           caller-owned device buffers (as hbam_sort_split): one ncclGroupStart of per-peer
 *           ncclSend / ncclRecv of keys, voffsets, block sizes and payload bytes (rank r gets
 *           the keys in (sp[r-1], sp[r]]), then hbam_sort_received on what arrived (chunks in
 *           source-rank order), so out is rank r's slice of the total order (key, file order).
 * A communicator is tied to one context (its device and stream). */
typedef struct hbam_comm hbam_comm;
#define HBAM_UNIQUE_ID_BYTES 128
int hbam_comm_unique_id(uint8_t* id_out);
int hbam_comm_init(hbam_ctx* ctx, const uint8_t* id, int32_t nranks, int32_t rank, hbam_comm** out);
void hbam_comm_destroy(hbam_comm* comm);
int hbam_comm_split_points(hbam_ctx* ctx, hbam_comm* comm, const hbam_sorted_run* run,
                           uint32_t samples_per_rank, int64_t* split_points);
int hbam_sort_exchange(hbam_ctx* ctx, hbam_comm* comm, const hbam_sorted_run* run,
                       const int64_t* split_points, hbam_sorted_run* out);

/* SplittingBAMIndexer (SplittingBAMIndexer.java:146-248, §8 f-2) from a whole-file decode
 * (dv: device columns of hbam_decode_split over [first record, len<<16|0xffff]): out (host)
 * = voffset of the first record, the voffset before every granularity-th record, then
 * file_len<<16 — the entries SplittingBAMIndex.java:50-77 reads (big-endian on disk).
 * Returns the entry count or a negative code. */
int64_t hbam_splitting_index(hbam_ctx* ctx, const hbam_columns* dv, int32_t granularity,
                             uint64_t file_len, uint64_t* out, uint64_t cap);
/* BGZFBlockIndexer.index (util/BGZFBlockIndexer.java:97-181, §8 f-3): the whole BGZF file
 * (host or device per on_device) -> out (host) = the compressed offset after every
 * granularity-th block, then the file length: the 48-bit values written big-endian as
 * [file].bgzfi and read by BGZFBlockIndex.java:50-69.  The indexer's `pos` is a Java int,
 * so entries past 2 GiB are the low 48 bits of the sign-extended wrapped value, as there.
 * Returns the entry count, HBAM_EIO where skipBlock raises IOException, or <0. */
int64_t hbam_bgzf_block_index(hbam_ctx* ctx, const uint8_t* file, int on_device, uint64_t len,
                              int32_t granularity, uint64_t* out, uint64_t cap);
/* out[i] = src[perm[i]] for elem_size 4 or 8 (device pointers): carries a column (voffset,
 * block_size) through a sort permutation. */
int hbam_permute(hbam_ctx* ctx, const void* src, uint32_t elem_size, const uint32_t* perm,
                 uint64_t n, void* out);

/* ---- BAM output ---------------------------------------------------------
 * hbam_bgzf_compress: [htsjdk] BlockCompressedOutputStream under BAMRecordWriter
 * (BAMRecordWriter.java:96-111, 113-124: the writer's stream, flushed without the EOF
 * terminator) and SAMOutputPreparer.prepareForRecords (util/SAMOutputPreparer.java:58-95).
 * Cuts [src, src + n) into blocks of block_size uncompressed bytes (0: 65280, at most 65280)
 * and writes one BGZF member per block (DEFLATE on the device, CRC32, ISIZE) back to back
 * into dst.  Returns the compressed length (>= 0) or a negative hbam status; dst_cap must be
 * at least hbam_bgzf_bound(n, block_size).  The compressed bytes are not zlib's: parity is
 * on the inflated bytes (any reader of BGZF gets src back).  No terminator is written: the
 * caller appends the 28-byte EOF block where the reference does (Utils.mergeSAMInto,
 * cli/Utils.java:351-353). */
uint64_t hbam_bgzf_bound(uint64_t n, uint32_t block_size);
int64_t hbam_bgzf_compress(hbam_ctx* ctx, const uint8_t* src, int src_on_device, uint64_t n,
                           uint32_t block_size, uint8_t* dst, int dst_on_device, uint64_t dst_cap);

/* ---- read-name / CIGAR keyed consumers -------------------------------------
 * Output buffers are device memory owned by the context, valid until the next call of the same
 * entry point on that context. */
/* SummarizeRecordReader (cli/plugins/chipster/Summarize.java:664-755) over a decoded split (dv:
 * device columns of hbam_decode_split / hbam_split_next): for every record that is mapped, placed
 * and has getAlignmentStart() >= 0 (:708-709), the reference ranges of its CIGAR (parseCIGAR
 * :719-755; M/=/X runs, D/N skip) in order, each with the LongWritable key nextKeyValue sets
 * (:696-699, :714-715: getKey0(refIdx, centre of mass), then the high word kept).  status: the
 * exception nextKeyValue raises after the n ranges — the split's own (dv->status), HBAM_EREFID
 * (IllegalArgumentException: a CIGAR op code > 8) or HBAM_EINDEX (a record without a range). */
typedef struct hbam_ranges {
  uint64_t n;
  int32_t status;
  int32_t pad;
  int64_t* key;
  int32_t* beg;      /* Range.beg: 1-based, inclusive */
  int32_t* end;      /* Range.end: inclusive */
  uint8_t* rev;      /* Range.reverseStrand */
  uint32_t* record;  /* the record (index in dv) the range comes from */
} hbam_ranges;
int hbam_summarize_ranges(hbam_ctx* ctx, const hbam_columns* dv, hbam_ranges* out);
/* FixMateMapper's shuffle (cli/plugins/FixMate.java:209-221): perm (device, u32[n]) = the n records
 * at ubuf + rec_off[i] (device; a decoded split's ubuf/rec_off or a packed payload and its offsets)
 * in the order of their Text(getReadName()) keys — unsigned lexicographic, proper prefix first —
 * ties in input order (the reference leaves them unspecified). */
int hbam_name_order(hbam_ctx* ctx, const uint8_t* ubuf, const uint64_t* rec_off, uint64_t n, uint32_t* perm);
/* FixMateReducer (FixMate.java:225-277) over that shuffle order, without the combiner: the
 * reducer's writes in order.  Output k is SAMRecordWritable.write of input record src[k] — as read
 * (mate[k] == 0xffffffff: a secondary, or an unpaired primary) or after SamPairUtil.setMateInfo with
 * record mate[k] (mate fields, flags 0x8/0x20, TLEN, MQ set / MC removed, re-encoded).  The
 * reducer's quirk is kept: a primary followed only by secondaries is mated with the last of them,
 * which is written twice.  status: HBAM_EFORMAT when a mated record's attributes do not parse (the
 * job fails at output n). */
typedef struct hbam_fixmate_run {
  uint64_t n;
  uint64_t payload_bytes;
  uint64_t n_groups;   /* reduce groups (distinct read names) */
  int32_t status;
  int32_t pad;
  uint32_t* src;
  uint32_t* mate;
  uint64_t* offsets;   /* n+1 */
  uint8_t* payload;
} hbam_fixmate_run;
int hbam_fixmate(hbam_ctx* ctx, const uint8_t* ubuf, const uint64_t* rec_off, uint64_t n,
                 hbam_fixmate_run* out);

/* ---- diagnostics (no reference counterpart) -----------------------------------------------
 * hbam_resolve_tokens: the LZ77 pass of the batched inflate (k_resolve) over ONE caller-built
 * token block: `io` (host, isize <= 65536 bytes) holds literal bytes with a 3-byte descriptor
 * (len-3, dist-1 little-endian) at the start of every match hole, `bitmap` (host,
 * ceil(isize/32) words) one bit per match start, tail_token/tail_dist the final match shorter
 * than 3 bytes (op | n<<16 | 1<<31, or 0).  On return `io` holds the resolved bytes and
 * *status is HBAM_OK, or HBAM_EDATA when a token points outside the block or has a distance
 * above DEFLATE's 32768 (the pass refuses such a block instead of copying from outside it). */
int hbam_resolve_tokens(hbam_ctx* ctx, uint8_t* io, uint32_t isize, const uint32_t* bitmap,
                        uint32_t tail_token, uint32_t tail_dist, int32_t* status);

/* ---- BCF over BGZF ---------------------------------------------------- */
/* BCF2Codec.readHeader: what the guesser and the record decode need from the header. */
typedef struct hbam_bcf_header {
  int32_t n_contig;       /* ##contig lines (BCF2Codec contigNames; CHROM indexes them) */
  int32_t n_sample;       /* header.getNGenotypeSamples() */
  int32_t n_dict;         /* string dictionary: PASS + FILTER/INFO/FORMAT IDs, first occurrence
                             (BCF2Utils.makeDictionary; whether htsjdk 1.131's shouldBeAddedToDictionary()
                             also admits ##ALT / ##contig lines is unverified: parity unpinned) */
  int32_t bgzf;           /* BlockCompressedInputStream.isValidFile(file) */
  uint64_t header_len;    /* uncompressed bytes of magic, l_text and the header text */
  uint64_t first_voffset; /* position of the first record: virtual offset (BGZF) or file offset */
} hbam_bcf_header;

/* BCFRecordReader output of one split (device memory owned by the context, valid until the
 * next call on it).  Record i's bytes are data[rec_off[i], +8 + l_shared + l_indiv). */
typedef struct hbam_bcf_columns {
  uint64_t n_records;
  int32_t status;       /* HBAM_OK, or the exception nextKeyValue() raises after n_records */
  int32_t pad0;
  uint64_t err_record;  /* == n_records */
  int64_t* rel;         /* BGZF: uncompressed bytes from the split start; plain: file offset */
  uint64_t* rec_off;    /* offset of the record's l_shared field in data */
  uint8_t* data;        /* the record stream: inflated blocks (BGZF) or the file window (plain) */
  uint64_t data_len;
  int64_t* key;         /* BCFRecordReader key: (long)contig index << 32 | (long)(start - 1) */
  int32_t* l_shared;
  int32_t* l_indiv;
  int32_t* chrom;
  int32_t* pos;         /* 0-based POS */
  int32_t* rlen;
  uint32_t* qual;       /* QUAL float bits */
  int32_t* n_allele_info;
  int32_t* n_fmt_sample;
} hbam_bcf_columns;

/* BCF2Codec.readHeader over the file's first `len` bytes (BGZF blocks inflated on the device).
 * HBAM_EMORE: the header runs past len.  Replaces BCFSplitGuesser.java:91-113 / BCFRecordReader
 * .initContigDict :125-133. */
int hbam_bcf_parse_header(hbam_ctx* ctx, const uint8_t* file, uint64_t len, hbam_bcf_header* out);

/* Bytes BCFSplitGuesser.guessNextBCFRecordStart(beg, end) reads (BCFSplitGuesser.java:133-145):
 * min((int)(end-beg), 2*0xffff+0xfffe) for BGZF, min(.., 0x80000) uncompressed, cut at EOF. */
uint64_t hbam_guess_bcf_window_len(uint64_t file_len, int64_t beg, int64_t end, int bgzf);

/* k guessNextBCFRecordStart calls over caller-gathered windows (window i =
 * windows[win_off[i], win_off[i+1]) = exactly hbam_guess_bcf_window_len bytes from beg[i]).
 * out[i]: virtual offset (BGZF) / file offset (plain) of the guessed record, or end[i];
 * err[i]: the exception escaping the guesser (HBAM_OK normally).  Replaces
 * BCFSplitGuesser.java:128-281 as called by VCFInputFormat.addGuessedSplits :269. */
int hbam_guess_bcf_windows(hbam_ctx* ctx, const uint8_t* windows, int on_device, const uint64_t* win_off,
                           uint64_t file_len, const int64_t* beg, const int64_t* end, uint64_t k,
                           const hbam_bcf_header* h, int64_t* out, int32_t* err);

/* BCFRecordReader over one split (BCFRecordReader.java:71-174): BGZF -> FileVirtualSplit
 * [v_start, v_end) read through BGZFLimitingStream (:177-237); plain -> FileSplit start =
 * v_start, length = v_end.  comp = file bytes [comp_base, file_len) (a BCF split reads to the
 * end of the file).  The record decode is a restated subset of htsjdk's BCF2Codec (parity
 * unpinned; oracle/hbam_oracle_bcf.c lists the rules). */
int hbam_bcf_decode_split(hbam_ctx* ctx, const uint8_t* comp, int on_device, uint64_t comp_base,
                          uint64_t comp_len, uint64_t file_len, const hbam_bcf_header* h, uint64_t v_start,
                          uint64_t v_end, hbam_bcf_columns* out);

#ifdef __cplusplus
}
#endif
#endif
