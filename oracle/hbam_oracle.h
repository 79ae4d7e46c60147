/* hbam_oracle.h — CPU restatement of Hadoop-BAM's BAM read path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline — never as the product path (the product is libhbam.so, HIP only).
 *
 * Parity status: the reference's arithmetic lives in htsjdk 1.131 (not vendored,
 * no JVM here).  Inflate/CRC are pinned to zlib 1.2.11 — the library the JDK's
 * java.util.zip.Inflater/CRC32 wrap — and to the reference's bgzf-terminator.bin.
 * Everything above inflate (BlockCompressedInputStream cursor semantics,
 * BAMRecordCodec.decode, BAMSplitGuesser, BAMInputFormat split construction,
 * BAMRecordReader.getKey/MurmurHash3) is a restatement of the Java sources cited
 * per function; the reference has no BAM tests or fixtures, so those parts are
 * "parity unpinned" beyond the committed self-generated goldens.
 */
#ifndef HBAM_ORACLE_H
#define HBAM_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Java exception classes the reference path can raise, as codes. */
enum {
  OR_OK = 0,
  OR_EIO = -1,        /* java.io.IOException (checked) */
  OR_ETRUNC = -2,     /* htsjdk FileTruncatedException */
  OR_EFORMAT = -3,    /* htsjdk SAMFormatException */
  OR_ERUNTIMEIO = -4, /* htsjdk RuntimeIOException (wrapped IOException) */
  OR_EEOF = -5,       /* htsjdk RuntimeEOFException */
  OR_EREFID = -6,     /* IllegalArgumentException (reference index not in dictionary) */
  OR_EDATA = -7,      /* RuntimeException wrapping java.util.zip.DataFormatException */
  OR_ENOMEM = -8,     /* host allocation failure (never modelled as OOM) */
  OR_ETRIBBLE = -14,  /* htsjdk TribbleException (BCF2Codec); = HBAM_ETRIBBLE */
  OR_ERUNTIME = -15   /* another RuntimeException escaping BCF2Codec.decode (unpinned); = HBAM_ERUNTIME */
};

/* MurmurHash3.murmurhash3(byte[], int) — util/MurmurHash3.java:32-102 */
int64_t or_murmurhash3(const uint8_t* key, int32_t len, int32_t seed);

/* BAMRecordReader.getKey(SAMRecord) for an undecoded BAM record — BAMRecordReader.java:66-106 */
int64_t or_get_key(int32_t ref_id, int32_t pos0, uint16_t flag, const uint8_t* var, int32_t var_len);

/* BGZF chain walk from offset 0 (BGZFBlockIndexer.skipBlock semantics, :130-181 and
 * htsjdk BCIS.readBlock framing).  Returns number of blocks, or a negative code when the
 * chain breaks; *bad_off receives the offending offset. */
int64_t or_scan_blocks(const uint8_t* f, uint64_t len, uint64_t* coff, uint32_t* clen,
                       uint32_t* isize, uint32_t* crc, uint64_t cap, uint64_t* bad_off);

/* BlockGunzipper.unzipBlock restated over zlib: header checks, raw inflate to exactly
 * ISIZE bytes, optional CRC32.  Returns OR_OK or an error code. */
int or_inflate_block(const uint8_t* blk, uint32_t blk_len, uint8_t* out, uint32_t out_cap,
                     uint32_t* out_len, int check_crc);

typedef struct or_header {
  int32_t l_text;
  int32_t n_ref;
  uint64_t header_ulen;   /* uncompressed bytes occupied by the BAM header */
  uint64_t first_voffset; /* getFilePointer() right after the header */
} or_header;

/* SAMHeaderReader.readSAMHeaderFrom restated for BAM (magic, l_text, text, n_ref, refs). */
int or_read_header(const uint8_t* f, uint64_t len, or_header* h);

/* Record sink used by the split reader: one call per emitted (key, record). */
typedef struct or_record {
  uint64_t voffset;   /* bci.getFilePointer() before decode (BAMRecordReader.java:173) */
  int32_t block_size;
  int32_t ref_id, pos;      /* pos is 0-based (BAM field) */
  uint8_t l_read_name, mapq;
  uint16_t bin, n_cigar, flag;
  int32_t l_seq, next_ref_id, next_pos, tlen;
  const uint8_t* var;       /* block_size-32 bytes: name, cigar, seq, qual, aux */
  int64_t key;
} or_record;

typedef int (*or_record_cb)(void* user, const or_record* r);

typedef struct or_read_result {
  uint64_t n_records;
  int32_t status;       /* OR_OK, or the exception nextKeyValue/initialize raised */
  uint64_t err_record;  /* index of the record being decoded when status was raised */
} or_read_result;

/* BAMRecordReader.initialize + nextKeyValue loop over one FileVirtualSplit
 * (BAMRecordReader.java:108-188).  check_crc mirrors BCIS.setCheckCrcs (off by default). */
int or_read_split(const uint8_t* f, uint64_t len, uint64_t v_start, uint64_t v_end,
                  int check_crc, or_record_cb cb, void* user, or_read_result* res);

/* BAMSplitGuesser.guessNextBAMRecordStart(beg, end) — BAMSplitGuesser.java:109-398.
 * n_ref = header dictionary size.  Returns the virtual offset or `end`.  *err receives
 * an exception code if one escapes the guesser (OR_OK otherwise). */
int64_t or_guess_bam_record_start(const uint8_t* f, uint64_t len, int64_t beg, int64_t end,
                                  int32_t n_ref, int* err);

/* BGZFSplitGuesser.guessNextBGZFBlockStart(beg, end) — util/BGZFSplitGuesser.java:51-148 */
int64_t or_guess_bgzf_block_start(const uint8_t* f, uint64_t len, int64_t beg, int64_t end,
                                  int* err);

/* Hadoop 1.2.1 FileInputFormat split sizing (SPLIT_SLOP 1.1), for one file. */
int64_t or_file_splits(uint64_t file_len, uint64_t split_size, uint64_t* beg, uint64_t* end,
                       uint64_t cap);

/* BAMInputFormat.addProbabilisticSplits for one file (BAMInputFormat.java:163-224).
 * Input: FileSplits [beg[i], end[i]).  Output: FileVirtualSplits (v_start, v_end).
 * Returns the number of virtual splits or a negative code (OR_EIO for "no reads in
 * first split"). */
int64_t or_probabilistic_splits(const uint8_t* f, uint64_t len, const uint64_t* beg,
                                const uint64_t* end, uint64_t n, uint64_t* v_start,
                                uint64_t* v_end);

/* SplittingBAMIndexer.index (SplittingBAMIndexer.java:146-186): voffset of the first
 * record, every granularity-th record, then file_len<<16.  Returns count or <0. */
int64_t or_splitting_index(const uint8_t* f, uint64_t len, int32_t granularity, uint64_t* out,
                           uint64_t cap);

/* BGZFBlockIndexer.index (util/BGZFBlockIndexer.java:97-181): compressed offset after every
 * granularity-th BGZF block (int `pos`, wraps past 2 GiB), then the file length.  Returns
 * the entry count or OR_EIO. */
int64_t or_bgzf_block_index(const uint8_t* f, uint64_t len, int32_t granularity, uint64_t* out,
                            uint64_t cap);

/* Columnar capture of or_read_split (for parity tests and the CPU baseline). */
typedef struct or_cols {
  uint64_t n;
  int32_t status;
  uint64_t err_record;
  uint64_t* voffset;
  int64_t* key;
  int32_t* block_size;
  int32_t* ref_id;
  int32_t* pos;
  uint8_t* l_read_name;
  uint8_t* mapq;
  uint16_t* bin;
  uint16_t* n_cigar;
  uint16_t* flag;
  int32_t* l_seq;
  int32_t* next_ref_id;
  int32_t* next_pos;
  int32_t* tlen;
  uint64_t* var_off; /* n+1 offsets into var */
  uint8_t* var;      /* concatenated variable blocks (block_size-32 bytes each) */
  uint64_t cap, var_cap;
} or_cols;

int or_read_split_cols(const uint8_t* f, uint64_t len, uint64_t v_start, uint64_t v_end,
                       int check_crc, int keep_var, or_cols* out);
/* the same with the header read elsewhere: f is a window of the file (a shard), n_ref >= 0 the
 * header's dictionary size (n_ref < 0: read the header from f, as or_read_split_cols) */
int or_read_split_cols_nref(const uint8_t* f, uint64_t len, uint64_t v_start, uint64_t v_end,
                            int check_crc, int keep_var, int32_t n_ref, or_cols* out);
void or_cols_free(or_cols* c);
/* CPU baseline (bench.py): the same read with the columns AND the lazy getters' pools the device
 * path materialises (names, CIGAR, SEQ characters, QUAL, AUX) built into host buffers, then freed.
 * *record_bytes = sum of block_size + 4; *pool_bytes = the pools' size. */
int or_read_split_pools(const uint8_t* f, uint64_t len, uint64_t v_start, uint64_t v_end, int32_t n_ref,
                        uint64_t* n_records, uint64_t* record_bytes, uint64_t* pool_bytes);

/* addProbabilisticSplits over a window of the file (a byte-range shard without the header):
 * the same as or_probabilistic_splits with the dictionary size given. */
int64_t or_probabilistic_splits_nref(const uint8_t* f, uint64_t len, const uint64_t* beg,
                                     const uint64_t* end, uint64_t n, int32_t n_ref,
                                     uint64_t* v_start, uint64_t* v_end);

/* ---- whole-output checker (bench.py's at-size parity; test infrastructure) ----------------
 * A decode's host copy (the device path's columns, pools and record bytes, record i at index i),
 * compared record by record with the oracle's read of one FileVirtualSplit: every fixed column,
 * the key, the voffset (+ voff_base), the record's variable bytes and every lazy-getter pool
 * (names incl. NUL, CIGAR u32s, SEQ as "=ACMGRSVTWYHKDBN" characters, QUAL, AUX, layout_ok).
 * The split's records are expected at device indices [first, first + n). */
typedef struct or_dev_cols {
  uint64_t n;
  uint64_t voff_base;
  const uint64_t* voffset;
  const int64_t* key;
  const uint64_t* rec_off;
  const uint8_t* ubuf;
  uint64_t ubuf_len;
  const int32_t *block_size, *ref_id, *pos;
  const uint8_t *l_read_name, *mapq;
  const uint16_t *bin, *n_cigar, *flag;
  const int32_t *l_seq, *next_ref_id, *next_pos, *tlen;
  const uint8_t* layout_ok;
  const uint64_t *name_off, *cigar_off, *seq_off, *aux_off; /* n+1; cigar_off counts u32s */
  const uint8_t* names;
  const uint32_t* cigars;
  const uint8_t *seq, *qual, *aux;
} or_dev_cols;

typedef struct or_check {
  uint64_t n_checked;    /* oracle records compared */
  uint64_t mismatches;   /* records that differ in any field */
  int64_t first_bad;     /* device index of the first differing record, -1 if none */
  int32_t bad_field;     /* which field differed first (see hbam_oracle.c: CK_*) */
  int32_t status;        /* the oracle read's status (0, or the exception it raised) */
} or_check;

int or_check_split(const uint8_t* f, uint64_t len, uint64_t v_start, uint64_t v_end, int32_t n_ref,
                   const or_dev_cols* dev, uint64_t first, or_check* out);


/* ---- read-name / CIGAR keyed consumers (hbam_oracle_f4.c) ----------------
 * Records are SAMRecordWritable payloads (block_size + record) at pay + off[i]. */
/* SummarizeRecordReader (cli/plugins/chipster/Summarize.java:664-755): ranges of every mapped
 * record; returns the count, *status = the exception raised after them (split_status, OR_EREFID
 * for a CIGAR op > 8, -13 IndexOutOfBoundsException for a record without a range). */
int64_t or_summarize_ranges(const uint8_t* pay, const uint64_t* off, uint64_t n, int32_t split_status,
                            int64_t* key, int32_t* beg, int32_t* end, uint8_t* rev, uint32_t* rec,
                            uint64_t cap, int32_t* status);
/* FixMateMapper's shuffle order: (Text(readName), input order) */
void or_name_order(const uint8_t* pay, const uint64_t* off, uint64_t n, uint32_t* perm);
/* FixMateReducer (FixMate.java:230-277) over the shuffle order: the reducer's writes */
int64_t or_fixmate(const uint8_t* pay, const uint64_t* off, uint64_t n, uint8_t* out_pay, uint64_t* out_off,
                   uint32_t* out_src, uint64_t cap, uint64_t pay_cap, int32_t* status);

/* ---- BCF, hbam_oracle_bcf.c ---------------------------------------- */
/* BCF2Codec.readHeader of uncompressed stream bytes: contig count, sample count, string
 * dictionary size, bytes of magic + l_text + text.  OR_EEOF: more bytes needed. */
int or_bcf_read_header(const uint8_t* u, uint64_t n, int32_t* n_contig, int32_t* n_sample,
                       int32_t* n_dict, uint64_t* header_len);
/* BCFSplitGuesser.guessNextBCFRecordStart (BCFSplitGuesser.java:128-281) over the whole file */
int64_t or_guess_bcf_record_start(const uint8_t* f, uint64_t len, int64_t beg, int64_t end, int is_bgzf,
                                  int32_t n_contig, int32_t n_sample, int32_t n_dict, int* err);
/* BCFRecordReader over one split (BGZF: FileVirtualSplit [v_start, v_end); uncompressed:
 * FileSplit start = v_start, length = v_end).  rel: record position (BGZF: uncompressed bytes
 * from the split start; uncompressed: file offset). */
int64_t or_read_bcf_split(const uint8_t* f, uint64_t len, int is_bgzf, uint64_t v_start, uint64_t v_end,
                          int32_t n_contig, int32_t n_sample, int32_t n_dict, uint64_t header_len,
                          int64_t* rel, int32_t* chrom, int32_t* pos, int64_t* key, uint64_t cap,
                          int* status);

#ifdef __cplusplus
}
#endif
#endif
