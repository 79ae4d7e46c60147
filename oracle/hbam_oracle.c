/* hbam_oracle.c — CPU restatement of Hadoop-BAM's BAM read path (TEST INFRASTRUCTURE).
 *
 * See hbam_oracle.h for the parity status.  Every function cites the reference
 * file:line it restates.  [htsjdk] marks behaviour of htsjdk 1.131 (pom.xml:43),
 * which is not vendored (3rdparty/htsjdk is an empty submodule): those parts restate
 * htsjdk's BlockCompressedInputStream / BlockGunzipper / BinaryCodec / BAMRecordCodec
 * as documented in SURVEY.md Appendix A.2-A.3.  Inflate and CRC32 are zlib itself,
 * the library java.util.zip wraps.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
 */
#define _GNU_SOURCE
#include "hbam_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <zlib.h>

/* ------------------------------------------------------------------------------ */
/* little-endian helpers (Java ByteBuffer LITTLE_ENDIAN)                            */
static inline int32_t rd_i32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24);
}
static inline uint16_t rd_u16(const uint8_t* p) { return (uint16_t)(p[0] | p[1] << 8); }
static inline int16_t rd_i16(const uint8_t* p) { return (int16_t)rd_u16(p); }
/* Java int arithmetic (wrapping) */
static inline int32_t jadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t jmul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

/* ------------------------------------------------------------------------------ */
/* MurmurHash3 — util/MurmurHash3.java:32-102, fmix :173-180                          */
static inline uint64_t rotl64(uint64_t x, int r) { return x << r | x >> (64 - r); }
static inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

int64_t or_murmurhash3(const uint8_t* key, int32_t len, int32_t seed) {
  const int32_t nblocks = len / 16;
  uint64_t h1 = (uint64_t)(int64_t)seed, h2 = (uint64_t)(int64_t)seed;
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  for (int32_t i = 0; i < nblocks; ++i) {
    uint64_t k1, k2;
    memcpy(&k1, key + 16 * i, 8);
    memcpy(&k2, key + 16 * i + 8, 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = h2 << 31 | h1 >> 33; /* MurmurHash3.java:59 — mixes h1, not rotl(h2,31) */
    h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* tail = key + 16 * nblocks;
  uint64_t k1 = 0, k2 = 0;
  switch (len & 15) {
    case 15: k2 ^= (uint64_t)tail[14] << 48; /* fallthrough */
    case 14: k2 ^= (uint64_t)tail[13] << 40; /* fallthrough */
    case 13: k2 ^= (uint64_t)tail[12] << 32; /* fallthrough */
    case 12: k2 ^= (uint64_t)tail[11] << 24; /* fallthrough */
    case 11: k2 ^= (uint64_t)tail[10] << 16; /* fallthrough */
    case 10: k2 ^= (uint64_t)tail[9] << 8;   /* fallthrough */
    case 9:
      k2 ^= (uint64_t)tail[8];
      k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
      /* fallthrough */
    case 8: k1 ^= (uint64_t)tail[7] << 56; /* fallthrough */
    case 7: k1 ^= (uint64_t)tail[6] << 48; /* fallthrough */
    case 6: k1 ^= (uint64_t)tail[5] << 40; /* fallthrough */
    case 5: k1 ^= (uint64_t)tail[4] << 32; /* fallthrough */
    case 4: k1 ^= (uint64_t)tail[3] << 24; /* fallthrough */
    case 3: k1 ^= (uint64_t)tail[2] << 16; /* fallthrough */
    case 2: k1 ^= (uint64_t)tail[1] << 8;  /* fallthrough */
    case 1:
      k1 ^= (uint64_t)tail[0];
      k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
      /* fallthrough */
    case 0: break;
  }
  h1 ^= (uint64_t)(int64_t)len;
  h2 ^= (uint64_t)(int64_t)len;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  return (int64_t)h1;
}

/* BAMRecordReader.getKey(SAMRecord) :66-96, getKey(int,int) :99-101, getKey0 :104-106.
 * The record is the lazily decoded BAMRecord, so getVariableBinaryRepresentation() is
 * the block_size-32 byte variable block. */
int64_t or_get_key(int32_t ref_id, int32_t pos0, uint16_t flag, const uint8_t* var, int32_t var_len) {
  const int32_t start = jadd(pos0, 1); /* getAlignmentStart() = pos+1 (int) */
  const int unmapped = (flag & 4) != 0;
  if (!(unmapped || ref_id < 0 || start < 0))
    return (int64_t)((uint64_t)(int64_t)ref_id << 32 | (uint64_t)(int64_t)jadd(start, -1));
  const int32_t hash = (int32_t)or_murmurhash3(var, var_len, 0);
  return (int64_t)((uint64_t)0x7fffffffULL << 32 | (uint64_t)(int64_t)hash);
}

/* ------------------------------------------------------------------------------ */
/* Seekable byte-array stream: util/SeekableArrayStream.java:29-58 (also used for the
 * whole file behind WrapSeekable: seek/read/eof have the same observable semantics). */
typedef struct ostream {
  const uint8_t* a;
  int64_t len;
  int64_t pos;
} ostream;

static int os_seek(ostream* s, int64_t p) { /* :40-45 */
  if (p < 0 || p > s->len) return OR_EIO;
  s->pos = p;
  return OR_OK;
}
static int32_t os_read(ostream* s, uint8_t* b, int32_t n) { /* :47-55 */
  if (s->pos == s->len) return -1;
  if ((int64_t)n > s->len - s->pos) n = (int32_t)(s->len - s->pos);
  memcpy(b, s->a + s->pos, (size_t)n);
  s->pos += n;
  return n;
}
static int os_eof(const ostream* s) { return s->pos == s->len; } /* :38 */

/* ------------------------------------------------------------------------------ */
/* [htsjdk] BlockGunzipper.unzipBlock over zlib.                     */
typedef struct gunzipper {
  z_stream z;
  int init;
} gunzipper;

static int gz_unzip(gunzipper* g, uint8_t* out, int32_t isize, const uint8_t* blk, int32_t blen,
                    int check_crc) {
  if (!(blk[0] == 0x1f && blk[1] == 0x8b && blk[2] == 8 && blk[3] == 4)) return OR_EFORMAT;
  if (rd_i16(blk + 10) != 6) return OR_EFORMAT;               /* XLEN */
  if ((int32_t)rd_u16(blk + 16) + 1 != blen) return OR_EFORMAT; /* BSIZE disagreement */
  const int32_t deflated = blen - 26;
  if (deflated < 0) return OR_EDATA; /* Inflater.setInput(b,18,<0): ArrayIndexOutOfBounds */
  const uint32_t expect_crc = (uint32_t)rd_i32(blk + 18 + deflated);
  if (!g->init) {
    memset(&g->z, 0, sizeof g->z);
    if (inflateInit2(&g->z, -15) != Z_OK) return OR_ENOMEM;
    g->init = 1;
  } else {
    inflateReset(&g->z);
  }
  uint8_t dummy = 0;
  g->z.next_in = (Bytef*)(blk + 18);
  g->z.avail_in = (uInt)deflated;
  g->z.next_out = isize > 0 ? out : &dummy;
  g->z.avail_out = (uInt)isize;
  /* java.util.zip.Inflater.inflate: one zlib inflate(Z_PARTIAL_FLUSH) call */
  int rc = inflate(&g->z, Z_PARTIAL_FLUSH);
  int32_t produced;
  if (rc == Z_DATA_ERROR) return OR_EDATA;          /* DataFormatException -> RuntimeException */
  if (rc == Z_MEM_ERROR) return OR_ENOMEM;
  if (rc == Z_BUF_ERROR) produced = 0;
  else produced = isize - (int32_t)g->z.avail_out;
  if (produced != isize) return OR_EFORMAT;         /* "Did not inflate expected amount" */
  if (check_crc) {
    uint32_t c = (uint32_t)crc32(0L, out, (uInt)isize);
    if (c != expect_crc) return OR_EFORMAT;         /* "CRC mismatch" */
  }
  return OR_OK;
}

int or_inflate_block(const uint8_t* blk, uint32_t blk_len, uint8_t* out, uint32_t out_cap,
                     uint32_t* out_len, int check_crc) {
  if (blk_len < 18 || blk_len > 65536) return OR_EIO;
  int32_t isize = rd_i32(blk + blk_len - 4);
  if (isize < 0) return OR_ERUNTIMEIO;
  if ((uint32_t)isize > out_cap) return OR_EFORMAT; /* cannot be produced by this caller */
  gunzipper g = {0};
  int rc = gz_unzip(&g, out, isize, blk, (int32_t)blk_len, check_crc);
  if (g.init) inflateEnd(&g.z);
  if (out_len) *out_len = (uint32_t)isize;
  return rc;
}

/* ------------------------------------------------------------------------------ */
/* [htsjdk] BlockCompressedInputStream: readBlock / inflateBlock /
 * available / read / seek / getFilePointer / eof.                                   */
#define BLOCK_HEADER_LENGTH 18
#define MAX_ISIZE_MODELLED (68u << 20) /* a <=64 KiB DEFLATE stream cannot exceed this */

typedef struct bcis {
  ostream* file;
  gunzipper gz;
  int check_crc;
  int64_t block_addr;  /* mBlockAddress */
  int32_t last_len;    /* mLastBlockLength */
  uint8_t* cur;        /* mCurrentBlock (NULL = null) */
  int32_t cur_len;
  int32_t cur_cap;
  int32_t cur_off;     /* mCurrentOffset */
  uint8_t fbuf[65536]; /* mFileBuffer */
} bcis;

static bcis* bcis_new(ostream* f, int check_crc) {
  bcis* b = (bcis*)calloc(1, sizeof(bcis));
  if (!b) return NULL;
  b->file = f;
  b->check_crc = check_crc;
  return b;
}
static void bcis_free(bcis* b) {
  if (!b) return;
  if (b->gz.init) inflateEnd(&b->gz.z);
  free(b->cur);
  free(b);
}
static int32_t bcis_read_bytes(bcis* b, uint8_t* buf, int32_t off, int32_t len) {
  int32_t n = 0;
  while (n < len) {
    int32_t c = os_read(b->file, buf + off + n, len - n);
    if (c <= 0) break;
    n += c;
  }
  return n;
}
static int bcis_set_block_len(bcis* b, int32_t len) {
  if (len > b->cur_cap) {
    uint8_t* p = (uint8_t*)realloc(b->cur, (size_t)(len > 0 ? len : 1));
    if (!p) return OR_ENOMEM;
    b->cur = p;
    b->cur_cap = len;
  }
  if (!b->cur) {
    b->cur = (uint8_t*)malloc(1);
    if (!b->cur) return OR_ENOMEM;
    b->cur_cap = 0;
  }
  b->cur_len = len;
  return OR_OK;
}
static int bcis_inflate_block(bcis* b, int32_t blen) {
  const int32_t isize = rd_i32(b->fbuf + blen - 4);
  /* mCurrentBlock = null before unzipping: a failed block leaves the cache empty */
  uint8_t* keep = b->cur;
  int32_t keep_cap = b->cur_cap;
  b->cur = NULL;
  b->cur_len = 0;
  b->cur_cap = 0;
  if (isize < 0) { free(keep); return OR_ERUNTIMEIO; } /* NegativeArraySizeException */
  if ((uint32_t)isize > MAX_ISIZE_MODELLED) { free(keep); return OR_EFORMAT; }
  b->cur = keep;
  b->cur_cap = keep_cap;
  int rc = bcis_set_block_len(b, isize);
  if (rc) return rc;
  rc = gz_unzip(&b->gz, b->cur, isize, b->fbuf, blen, b->check_crc);
  if (rc) {
    b->cur_len = -1; /* sentinel: mCurrentBlock == null (buffer kept for reuse) */
    return rc;
  }
  return OR_OK;
}
#define CUR_IS_NULL(b) ((b)->cur == NULL || (b)->cur_len < 0)

static int bcis_read_block(bcis* b) {
  int32_t count = bcis_read_bytes(b, b->fbuf, 0, BLOCK_HEADER_LENGTH);
  if (count == 0) { /* no empty gzip block at end */
    b->cur_off = 0;
    b->block_addr += b->last_len;
    int rc = bcis_set_block_len(b, 0);
    return rc;
  }
  if (count != BLOCK_HEADER_LENGTH) return OR_EIO; /* "Premature end of file" */
  const int32_t blen = (int32_t)rd_u16(b->fbuf + 16) + 1;
  if (blen < BLOCK_HEADER_LENGTH || blen > 65536) return OR_EIO;
  const int32_t remaining = blen - BLOCK_HEADER_LENGTH;
  count = bcis_read_bytes(b, b->fbuf, BLOCK_HEADER_LENGTH, remaining);
  if (count != remaining) return OR_ETRUNC;
  int rc = bcis_inflate_block(b, blen);
  if (rc) return rc;
  b->cur_off = 0;
  b->block_addr += b->last_len;
  b->last_len = blen;
  return OR_OK;
}
/* available(): one readBlock when the current block is exhausted (1.131 behaviour:
 * an empty block therefore reads as end-of-stream for that one read call). */
static int bcis_available(bcis* b, int32_t* avail) {
  if (CUR_IS_NULL(b) || b->cur_off == b->cur_len) {
    int rc = bcis_read_block(b);
    if (rc) return rc;
  }
  *avail = CUR_IS_NULL(b) ? 0 : b->cur_len - b->cur_off;
  return OR_OK;
}
/* read(byte[],int,int): returns bytes copied, -1 at EOF (nothing copied). */
static int bcis_read(bcis* b, uint8_t* buf, int32_t len, int32_t* got) {
  const int32_t orig = len;
  int32_t off = 0;
  while (len > 0) {
    int32_t avail;
    int rc = bcis_available(b, &avail);
    if (rc) return rc;
    if (avail == 0) {
      if (orig == len) { *got = -1; return OR_OK; }
      break;
    }
    int32_t c = len < avail ? len : avail;
    memcpy(buf + off, b->cur + b->cur_off, (size_t)c);
    b->cur_off += c;
    off += c;
    len -= c;
  }
  *got = orig - len;
  return OR_OK;
}
static int bcis_eof(bcis* b) {
  if (os_eof(b->file)) return 1;
  return b->file->len - (b->block_addr + b->last_len) == 28; /* EMPTY_GZIP_BLOCK.length */
}
static int bcis_seek(bcis* b, uint64_t pos) {
  const int64_t coff = (int64_t)(pos >> 16);
  const int32_t uoff = (int32_t)(pos & 0xffff);
  int32_t avail;
  if (b->block_addr == coff && !CUR_IS_NULL(b)) {
    avail = b->cur_len;
  } else {
    int rc = os_seek(b->file, coff);
    if (rc) return rc;
    b->block_addr = coff;
    b->last_len = 0;
    rc = bcis_read_block(b);
    if (rc) return rc;
    rc = bcis_available(b, &avail);
    if (rc) return rc;
  }
  if (uoff > avail || (uoff == avail && !bcis_eof(b))) return OR_EIO; /* Invalid file pointer */
  b->cur_off = uoff;
  return OR_OK;
}
static uint64_t bcis_tell(const bcis* b) { /* getFilePointer() */
  if (b->cur_off == b->cur_len)
    return (uint64_t)(b->block_addr + b->last_len) << 16;
  return (uint64_t)b->block_addr << 16 | (uint64_t)(uint32_t)b->cur_off;
}

/* [htsjdk] BinaryCodec.readBytes: loop of read() calls; -1 -> RuntimeEOFException,
 * IOException -> RuntimeIOException. */
static int codec_read_bytes(bcis* b, uint8_t* buf, int32_t len) {
  int32_t total = 0;
  do {
    int32_t got;
    int rc = bcis_read(b, buf + total, len - total, &got);
    if (rc == OR_EIO) return OR_ERUNTIMEIO;
    if (rc) return rc;
    if (got < 0) return OR_EEOF;
    total += got;
  } while (total < len);
  return OR_OK;
}

/* Scratch used to discard bytes of an implausibly long record without holding them. */
typedef struct decoded {
  int32_t block_size, ref_id, pos, l_seq, next_ref_id, next_pos, tlen;
  uint8_t l_read_name, mapq;
  uint16_t bin, n_cigar, flag;
  uint8_t* var;
  int32_t var_cap;
} decoded;

/* [htsjdk] BAMRecordCodec.decode.  Returns 1 (record), 0 (null) or <0.
 * n_ref >= 0: default factory with a header (refID/mate refID validated,
 * IllegalArgumentException); n_ref < 0: LazyBAMRecordFactory (LazyBAMRecordFactory.java:31-99),
 * no validation.  A huge block_size is modelled as "allocation succeeds". */
static int codec_decode(bcis* b, int32_t n_ref, decoded* d) {
  uint8_t t[4];
  int rc = codec_read_bytes(b, t, 4);
  if (rc == OR_EEOF) return 0;
  if (rc) return rc;
  d->block_size = rd_i32(t);
  if (d->block_size < 32) return OR_EFORMAT; /* "Invalid record length" */
#define RD(n)                                  \
  do {                                         \
    rc = codec_read_bytes(b, t, (n));          \
    if (rc) return rc;                         \
  } while (0)
  RD(4); d->ref_id = rd_i32(t);
  RD(4); d->pos = rd_i32(t);
  RD(1); d->l_read_name = t[0];
  RD(1); d->mapq = t[0];
  RD(2); d->bin = rd_u16(t);
  RD(2); d->n_cigar = rd_u16(t);
  RD(2); d->flag = rd_u16(t);
  RD(4); d->l_seq = rd_i32(t);
  RD(4); d->next_ref_id = rd_i32(t);
  RD(4); d->next_pos = rd_i32(t);
  RD(4); d->tlen = rd_i32(t);
#undef RD
  const int32_t vlen = d->block_size - 32;
  if (vlen > d->var_cap) {
    /* grow geometrically but cap physical allocation; reads beyond the cap are
       streamed through a window (the record can only complete if the data exists) */
    int32_t want = vlen;
    uint8_t* p = (uint8_t*)realloc(d->var, (size_t)want);
    if (!p) return OR_ENOMEM;
    d->var = p;
    d->var_cap = want;
  }
  if (vlen > 0) {
    rc = codec_read_bytes(b, d->var, vlen);
    if (rc) return rc;
  }
  if (n_ref >= 0) { /* BAMRecord ctor: setReferenceIndex / setMateReferenceIndex */
    if (d->ref_id != -1 && (d->ref_id < 0 || d->ref_id >= n_ref)) return OR_EREFID;
    if (d->next_ref_id != -1 && (d->next_ref_id < 0 || d->next_ref_id >= n_ref)) return OR_EREFID;
  }
  return 1;
}

/* ------------------------------------------------------------------------------ */
/* BGZF chain walk: util/BGZFBlockIndexer.java:130-181 (skipBlock) with [htsjdk]
 * readBlock framing (BSIZE at offset 16, length BSIZE+1, ISIZE/CRC in the footer). */
int64_t or_scan_blocks(const uint8_t* f, uint64_t len, uint64_t* coff, uint32_t* clen,
                       uint32_t* isize, uint32_t* crc, uint64_t cap, uint64_t* bad_off) {
  uint64_t p = 0, n = 0;
  while (p < len) {
    if (len - p < 18 || !(f[p] == 0x1f && f[p + 1] == 0x8b && f[p + 2] == 8 && f[p + 3] == 4) ||
        rd_u16(f + p + 10) != 6 || f[p + 12] != 'B' || f[p + 13] != 'C' ||
        rd_u16(f + p + 14) != 2) {
      if (bad_off) *bad_off = p;
      return OR_EFORMAT;
    }
    uint32_t bl = (uint32_t)rd_u16(f + p + 16) + 1;
    if (bl < 26 || p + bl > len) {
      if (bad_off) *bad_off = p;
      return OR_ETRUNC;
    }
    if (n < cap) {
      coff[n] = p;
      clen[n] = bl;
      isize[n] = (uint32_t)rd_i32(f + p + bl - 4);
      crc[n] = (uint32_t)rd_i32(f + p + bl - 8);
    }
    ++n;
    p += bl;
  }
  return (int64_t)n;
}

/* ------------------------------------------------------------------------------ */
/* [htsjdk] SAMTextHeaderCodec.parseSQLine under STRICT stringency (the reader's default): the @SQ
 * lines of the text, in order, with their SN value and LN.  An @SQ line without SN or LN, or an LN
 * Integer.parseInt rejects, raises (returns -1).  Returns the number of @SQ lines. */
typedef struct sq_entry {
  const uint8_t* name;
  int32_t name_len;
  int32_t len;
} sq_entry;

static int32_t text_sq(const uint8_t* t, int32_t n, sq_entry** out) {
  int32_t cnt = 0, cap = 0;
  *out = NULL;
  for (int32_t a = 0; a < n;) {
    int32_t e = a;
    while (e < n && t[e] != '\n') ++e;
    int32_t z = e;
    if (z > a && t[z - 1] == '\r') --z; /* StringLineReader: "\r\n" ends a line */
    if (z - a >= 3 && memcmp(t + a, "@SQ", 3) == 0 && (z - a == 3 || t[a + 3] == '\t')) {
      sq_entry x = {NULL, 0, 0};
      int has_sn = 0, has_ln = 0;
      for (int32_t f = a + 3; f < z;) { /* tab-separated TAG:value fields */
        int32_t g = f + 1;
        while (g < z && t[g] != '\t') ++g;
        const uint8_t* v = t + f + 1;
        const int32_t vl = g - f - 1;
        if (vl >= 3 && v[2] == ':' && v[0] == 'S' && v[1] == 'N' && !has_sn) {
          x.name = v + 3;
          x.name_len = vl - 3;
          has_sn = 1;
        } else if (vl >= 3 && v[2] == ':' && v[0] == 'L' && v[1] == 'N' && !has_ln) {
          int32_t k = 3, neg = 0;
          int64_t ln = 0;
          if (k < vl && (v[k] == '-' || v[k] == '+')) neg = v[k++] == '-';
          if (k == vl) { free(*out); *out = NULL; return -1; }
          for (; k < vl; ++k) {
            if (v[k] < '0' || v[k] > '9' || (ln = ln * 10 + (v[k] - '0')) > 2147483648LL) { free(*out); *out = NULL; return -1; }
          }
          if (neg) ln = -ln;
          if (ln > 2147483647LL) { free(*out); *out = NULL; return -1; }
          x.len = (int32_t)ln;
          has_ln = 1;
        }
        f = g;
      }
      if (!has_sn || !has_ln) { free(*out); *out = NULL; return -1; }
      if (cnt == cap) {
        cap = cap ? 2 * cap : 64;
        sq_entry* np = (sq_entry*)realloc(*out, (size_t)cap * sizeof *np);
        if (!np) { free(*out); *out = NULL; return -1; }
        *out = np;
      }
      (*out)[cnt++] = x;
    }
    a = e + 1;
  }
  return cnt;
}

/* SAMHeaderReader.readSAMHeaderFrom (util/SAMHeaderReader.java:53-72) for BAM:
 * [htsjdk] BAMFileReader.readHeader — magic, l_text, text, n_ref, {l_name,name,l_ref}.  When the
 * text holds @SQ lines the binary dictionary must match them: the count (checked before any
 * entry is read), then per entry the name (the binary one cut at its first whitespace,
 * SAMSequenceUtil.truncateSequenceName) and the length; readSequenceRecord rejects l_name <= 1
 * ("missing sequence name").  All SAMFormatException.  Restated from htsjdk 1.131's published
 * source (absent here: parity unpinned). */
int or_read_header(const uint8_t* f, uint64_t len, or_header* h) {
  ostream s = {f, (int64_t)len, 0};
  bcis* b = bcis_new(&s, 0);
  if (!b) return OR_ENOMEM;
  int rc;
  uint8_t t[4];
  uint8_t* text = NULL;
  uint8_t* name = NULL;
  sq_entry* sq = NULL;
  int32_t nsq = 0;
#define HR(buf, n)                                   \
  do {                                               \
    rc = codec_read_bytes(b, (buf), (n));            \
    if (rc) goto out;                                \
  } while (0)
  HR(t, 4);
  if (memcmp(t, "BAM\1", 4) != 0) { rc = OR_EFORMAT; goto out; }
  HR(t, 4);
  h->l_text = rd_i32(t);
  if (h->l_text < 0) { rc = OR_EFORMAT; goto out; }
  text = (uint8_t*)malloc((size_t)h->l_text + 1);
  if (!text) { rc = OR_ENOMEM; goto out; }
  if (h->l_text) HR(text, h->l_text);
  nsq = text_sq(text, h->l_text, &sq);
  if (nsq < 0) { rc = OR_EFORMAT; goto out; }
  HR(t, 4);
  h->n_ref = rd_i32(t);
  if (h->n_ref < 0) { rc = OR_EFORMAT; goto out; }
  if (nsq > 0 && nsq != h->n_ref) { rc = OR_EFORMAT; goto out; }
  uint64_t ulen = 12 + (uint64_t)h->l_text;
  for (int32_t i = 0; i < h->n_ref; ++i) {
    HR(t, 4);
    int32_t ln = rd_i32(t);
    if (ln <= 1) { rc = OR_EFORMAT; goto out; }
    free(name);
    name = (uint8_t*)malloc((size_t)ln);
    if (!name) { rc = OR_ENOMEM; goto out; }
    HR(name, ln);
    HR(t, 4);
    if (nsq > 0) {
      int32_t k = 0;
      while (k < ln - 1 && !(name[k] == ' ' || (name[k] >= 9 && name[k] <= 13))) ++k;
      if (sq[i].name_len != k || memcmp(sq[i].name, name, (size_t)k) != 0) { rc = OR_EFORMAT; goto out; }
      if (sq[i].len != rd_i32(t)) { rc = OR_EFORMAT; goto out; }
    }
    ulen += 8 + (uint64_t)ln;
  }
  h->header_ulen = ulen;
  h->first_voffset = bcis_tell(b);
  rc = OR_OK;
out:
#undef HR
  if (rc == OR_EEOF || rc == OR_ERUNTIMEIO) rc = OR_EFORMAT;
  free(text);
  free(name);
  free(sq);
  bcis_free(b);
  return rc;
}

/* ------------------------------------------------------------------------------ */
/* BAMRecordReader.initialize (:108-151) + nextKeyValue (:172-188).                  */
static int read_split_body(const uint8_t* f, uint64_t len, uint64_t v_start, uint64_t v_end,
                           int check_crc, int32_t n_ref, or_record_cb cb, void* user, or_read_result* res);
int or_read_split(const uint8_t* f, uint64_t len, uint64_t v_start, uint64_t v_end,
                  int check_crc, or_record_cb cb, void* user, or_read_result* res) {
  memset(res, 0, sizeof *res);
  or_header h;
  int rc = or_read_header(f, len, &h);
  if (rc) { res->status = rc; return rc; }
  return read_split_body(f, len, v_start, v_end, check_crc, h.n_ref, cb, user, res);
}

/* The same loop when the header was read elsewhere (BAMRecordReader.initialize reads it from the
 * start of the file, :128-130): f is a window of the file holding the split's blocks (a shard of a
 * byte-range-sharded file), voffsets relative to the window, n_ref the header's dictionary size. */
static int read_split_body(const uint8_t* f, uint64_t len, uint64_t v_start, uint64_t v_end,
                           int check_crc, int32_t n_ref, or_record_cb cb, void* user, or_read_result* res) {
  int rc;
  memset(res, 0, sizeof *res);
  struct { int32_t n_ref; } h = {n_ref};
  ostream s = {f, (int64_t)len, 0};
  bcis* b = bcis_new(&s, check_crc);
  if (!b) { res->status = OR_ENOMEM; return OR_ENOMEM; }
  rc = bcis_seek(b, v_start);
  if (rc) {
    res->status = rc;
    bcis_free(b);
    return rc;
  }
  decoded d;
  memset(&d, 0, sizeof d);
  for (;;) {
    const uint64_t fp = bcis_tell(b);
    if ((int64_t)fp >= (int64_t)v_end) break;
    rc = codec_decode(b, h.n_ref, &d);
    if (rc == 0) break;
    if (rc < 0) {
      res->status = rc;
      res->err_record = res->n_records;
      break;
    }
    or_record r;
    r.voffset = fp;
    r.block_size = d.block_size;
    r.ref_id = d.ref_id;
    r.pos = d.pos;
    r.l_read_name = d.l_read_name;
    r.mapq = d.mapq;
    r.bin = d.bin;
    r.n_cigar = d.n_cigar;
    r.flag = d.flag;
    r.l_seq = d.l_seq;
    r.next_ref_id = d.next_ref_id;
    r.next_pos = d.next_pos;
    r.tlen = d.tlen;
    r.var = d.var;
    r.key = or_get_key(d.ref_id, d.pos, d.flag, d.var, d.block_size - 32);
    ++res->n_records;
    if (cb && cb(user, &r)) break;
  }
  free(d.var);
  bcis_free(b);
  return res->status;
}

/* ------------------------------------------------------------------------------ */
/* BAMSplitGuesser — BAMSplitGuesser.java:77-398.                   */
#define BGZF_MAGIC 0x04088b1f
#define BGZF_MAGIC_SUB 0x00024342
#define BGZF_SUB_SIZE 6
#define BLOCKS_NEEDED_FOR_GUESS 3
#define MAX_BYTES_READ (BLOCKS_NEEDED_FOR_GUESS * 0xffff + 0xfffe)
#define SHORTEST_POSSIBLE_BAM_RECORD (4 * 9 + 1 + 1 + 1)

typedef struct guesser {
  const uint8_t* file;
  int64_t flen;
  int32_t n_ref;
  uint8_t buf[8]; /* ByteBuffer.allocate(8): persists across guesses (stale bytes) */
  ostream in;
  bcis* bgzf;
  decoded d;
} guesser;

static int32_t g_buf_i32(const guesser* g, int i) { return rd_i32(g->buf + i); }
static int32_t g_ushort(const guesser* g, int i) { return (int32_t)rd_u16(g->buf + i); }

/* guessNextBGZFPos :222-299.  Returns 1 with (pos,size) or 0 (null). */
static int g_next_bgzf(guesser* g, int32_t p, int32_t end, int32_t* opos, int32_t* osize) {
  ostream* in = &g->in;
  for (;;) {
    for (;;) {
      if (os_seek(in, p)) return 0;
      os_read(in, g->buf, 4);
      const int32_t n = g_buf_i32(g, 0);
      if (n == BGZF_MAGIC) break;
      if ((int32_t)((uint32_t)n >> 8) == (int32_t)(((uint32_t)BGZF_MAGIC << 8) >> 8)) ++p;
      else if ((int32_t)((uint32_t)n >> 16) == (int32_t)(((uint32_t)BGZF_MAGIC << 16) >> 16)) p += 2;
      else p += 3;
      if (p >= end) return 0;
    }
    const int32_t p0 = p;
    p += 10;
    if (os_seek(in, p)) return 0;
    os_read(in, g->buf, 2);
    p += 2;
    const int32_t xlen = g_ushort(g, 0);
    const int32_t sub_end = p + xlen;
    while (p < sub_end) {
      os_read(in, g->buf, 4);
      if (g_buf_i32(g, 0) != BGZF_MAGIC_SUB) {
        p += 4 + g_ushort(g, 2);
        if (os_seek(in, p)) return 0;
        continue;
      }
      os_read(in, g->buf, 2);
      const int32_t bsize = g_ushort(g, 0);
      p += BGZF_SUB_SIZE;
      while (p < sub_end) {
        if (os_seek(in, p)) return 0;
        os_read(in, g->buf, 4);
        p += 4 + g_ushort(g, 2);
      }
      if (p != sub_end) break;
      p += bsize - xlen - 19 + 4;
      if (os_seek(in, p)) return 0;
      os_read(in, g->buf, 4);
      *opos = p0;
      *osize = g_buf_i32(g, 0);
      return 1;
    }
    p = p0 + 4;
  }
}

/* guessNextBAMPos :301-398.  Returns the candidate or -1. */
static int32_t g_next_bam(guesser* g, uint64_t cp_virt, int32_t up, int32_t csize) {
  bcis* bz = g->bgzf;
  int32_t got;
  up += 4;
  while (up + SHORTEST_POSSIBLE_BAM_RECORD - 4 < csize) {
    if (bcis_seek(bz, cp_virt | (uint32_t)up)) return -1;
    if (bcis_read(bz, g->buf, 8, &got)) return -1;
    const int32_t id = g_buf_i32(g, 0), pos = g_buf_i32(g, 4);
    if (id < -1 || id > g->n_ref || pos < -1) { ++up; continue; }
    if (bcis_seek(bz, cp_virt | (uint32_t)(up + 20))) return -1;
    if (bcis_read(bz, g->buf, 8, &got)) return -1;
    const int32_t nid = g_buf_i32(g, 0), npos = g_buf_i32(g, 4);
    if (nid < -1 || nid > g->n_ref || npos < -1) { ++up; continue; }
    const int32_t next_up = up + 1;
    up -= 4;
    if (bcis_seek(bz, cp_virt | (uint32_t)(up + 12))) return -1;
    if (bcis_read(bz, g->buf, 4, &got)) return -1;
    const int32_t name_len = g_buf_i32(g, 0) & 0xff;
    const int32_t nul = up + 36 + name_len - 1;
    if (nul >= csize) { up = next_up; continue; }
    if (bcis_seek(bz, cp_virt | (uint32_t)nul)) return -1;
    if (bcis_read(bz, g->buf, 1, &got)) return -1;
    if (g->buf[0] != 0) { up = next_up; continue; }
    int32_t zero_min = 4 * 8 + name_len;
    if (bcis_seek(bz, cp_virt | (uint32_t)(up + 16))) return -1;
    if (bcis_read(bz, g->buf, 8, &got)) return -1;
    zero_min = jadd(zero_min, jmul(g_buf_i32(g, 0) & 0xffff, 4));
    const int32_t l_seq = g_buf_i32(g, 4);
    zero_min = jadd(zero_min, jadd(l_seq, jadd(l_seq, 1) / 2));
    if (bcis_seek(bz, cp_virt | (uint32_t)up)) return -1;
    if (bcis_read(bz, g->buf, 4, &got)) return -1;
    if (g_buf_i32(g, 0) < zero_min) { up = next_up; continue; }
    return up;
  }
  return -1;
}

/* guessNextBAMRecordStart :109-212 */
static int64_t g_guess(guesser* g, int64_t beg, int64_t end, int* err) {
  *err = OR_OK;
  /* buffer the window: loop of inFile.read calls (:116-125) */
  int32_t want = (int32_t)(end - beg);
  if (want > MAX_BYTES_READ) want = MAX_BYTES_READ;
  int64_t total = 0;
  if (want > 0 && beg >= 0 && beg <= g->flen) {
    total = g->flen - beg < want ? g->flen - beg : want;
  }
  g->in.a = g->file + (beg >= 0 && beg <= g->flen ? beg : 0);
  g->in.len = total;
  g->in.pos = 0;
  bcis_free(g->bgzf);
  g->bgzf = bcis_new(&g->in, 1); /* setCheckCrcs(true) */
  if (!g->bgzf) { *err = OR_ENOMEM; return end; }
  int32_t first_end = (int32_t)(end - beg);
  if (first_end > 0xffff) first_end = 0xffff;

  for (int32_t cp = 0;; ++cp) {
    int32_t psz_pos, psz_size;
    if (!g_next_bgzf(g, cp, first_end, &psz_pos, &psz_size)) return end;
    const int32_t cp0 = cp = psz_pos;
    const uint64_t cp0_virt = (uint64_t)(uint32_t)cp0 << 16;
    if (bcis_seek(g->bgzf, cp0_virt)) continue; /* catch (Throwable) */
    for (int32_t up = 0;; ++up) {
      const int32_t up0 = up = g_next_bam(g, cp0_virt, up, psz_size);
      if (up0 < 0) break;
      if (bcis_seek(g->bgzf, cp0_virt | (uint32_t)up0)) {
        /* seek inside the already-validated block cannot fail; treat like the
           reference would (IOException escapes the method) */
        *err = OR_EIO;
        return end;
      }
      int decoded_any = 0;
      int b = 0;
      int32_t prev_cp = cp0;
      int rc = 0;
      while (b < BLOCKS_NEEDED_FOR_GUESS) {
        rc = codec_decode(g->bgzf, -1, &g->d);
        if (rc <= 0) break;
        decoded_any = 1;
        const int32_t cp2 = (int32_t)(bcis_tell(g->bgzf) >> 16);
        if (cp2 != prev_cp) { prev_cp = cp2; ++b; }
      }
      if (rc < 0) {
        if (rc == OR_EFORMAT || rc == OR_ETRUNC || rc == OR_ENOMEM || rc == OR_EREFID ||
            rc == OR_ERUNTIMEIO)
          continue; /* :194-198 */
        if (rc == OR_EEOF) {
          if (!decoded_any && os_eof(&g->in)) continue; /* :199-207 */
        } else {
          *err = rc; /* RuntimeException / IOException escapes guessNextBAMRecordStart */
          return end;
        }
      } else if (b < BLOCKS_NEEDED_FOR_GUESS) {
        if (!decoded_any) continue; /* :188-192 */
      }
      return (int64_t)((uint64_t)(beg + cp0) << 16 | (uint32_t)up0);
    }
  }
}

static guesser* guesser_new(const uint8_t* f, uint64_t len, int32_t n_ref) {
  guesser* g = (guesser*)calloc(1, sizeof(guesser));
  if (!g) return NULL;
  g->file = f;
  g->flen = (int64_t)len;
  g->n_ref = n_ref;
  /* ctor :77-88: ss.seek(0); ss.read(buf, 0, 4) leaves the file magic in buf */
  for (int i = 0; i < 4 && (uint64_t)i < len; ++i) g->buf[i] = f[i];
  return g;
}
static void guesser_free(guesser* g) {
  if (!g) return;
  bcis_free(g->bgzf);
  free(g->d.var);
  free(g);
}

int64_t or_guess_bam_record_start(const uint8_t* f, uint64_t len, int64_t beg, int64_t end,
                                  int32_t n_ref, int* err) {
  guesser* g = guesser_new(f, len, n_ref);
  if (!g) { *err = OR_ENOMEM; return end; }
  int64_t r = g_guess(g, beg, end, err);
  guesser_free(g);
  return r;
}

/* ------------------------------------------------------------------------------ */
/* BGZFSplitGuesser.guessNextBGZFBlockStart — util/BGZFSplitGuesser.java:51-148.     */
int64_t or_guess_bgzf_block_start(const uint8_t* f, uint64_t len, int64_t beg, int64_t end,
                                  int* err) {
  *err = OR_OK;
  int32_t want = (int32_t)(end - beg);
  if (want > 2 * 0xffff - 1) want = 2 * 0xffff - 1;
  int64_t total = 0;
  if (want > 0 && beg >= 0 && beg <= (int64_t)len)
    total = (int64_t)len - beg < want ? (int64_t)len - beg : want;
  /* single read() call (:62-63); for an in-memory file it returns everything asked */
  ostream in = {f + (beg >= 0 && beg <= (int64_t)len ? beg : 0), total, 0};
  bcis* bz = bcis_new(&in, 1);
  if (!bz) { *err = OR_ENOMEM; return end; }
  uint8_t buf[8] = {0};
  int32_t first_end = (int32_t)(end - beg);
  if (first_end > 0xffff) first_end = 0xffff;
  int64_t result = end;
  for (int32_t pos = 0;;) {
    /* guessNextBGZFPos :95-148 (IOExceptions propagate from this variant) */
    int32_t p = pos;
    int found = 0;
    for (;;) {
      for (;;) {
        if (os_seek(&in, p)) { *err = OR_EIO; goto done; }
        os_read(&in, buf, 4);
        const int32_t n = rd_i32(buf);
        if (n == BGZF_MAGIC) break;
        if ((int32_t)((uint32_t)n >> 8) == (int32_t)(((uint32_t)BGZF_MAGIC << 8) >> 8)) ++p;
        else if ((int32_t)((uint32_t)n >> 16) == (int32_t)(((uint32_t)BGZF_MAGIC << 16) >> 16)) p += 2;
        else p += 3;
        if (p >= first_end) goto notfound;
      }
      const int32_t p0 = p;
      p += 10;
      if (os_seek(&in, p)) { *err = OR_EIO; goto done; }
      os_read(&in, buf, 2);
      p += 2;
      const int32_t xlen = (int32_t)rd_u16(buf);
      const int32_t sub_end = p + xlen;
      while (p < sub_end) {
        os_read(&in, buf, 4);
        if (rd_i32(buf) != BGZF_MAGIC_SUB) {
          p += 4 + (int32_t)rd_u16(buf + 2);
          if (os_seek(&in, p)) { *err = OR_EIO; goto done; }
          continue;
        }
        pos = p0;
        found = 1;
        break;
      }
      if (found) break;
      p = p0 + 4;
    }
    if (bcis_seek(bz, (uint64_t)(uint32_t)pos << 16)) { ++pos; continue; }
    result = beg + pos;
    goto done;
  notfound:
    result = end;
    goto done;
  }
done:
  bcis_free(bz);
  return result;
}

/* ------------------------------------------------------------------------------ */
/* Hadoop 1.2.1 FileInputFormat.getSplits for one file.             */
int64_t or_file_splits(uint64_t file_len, uint64_t split_size, uint64_t* beg, uint64_t* end,
                       uint64_t cap) {
  if (split_size == 0) return OR_EIO;
  uint64_t n = 0, rem = file_len;
  while ((double)rem / (double)split_size > 1.1) {
    if (n < cap) { beg[n] = file_len - rem; end[n] = file_len - rem + split_size; }
    ++n;
    rem -= split_size;
  }
  if (rem != 0) {
    if (n < cap) { beg[n] = file_len - rem; end[n] = file_len; }
    ++n;
  }
  return (int64_t)n;
}

/* BAMInputFormat.addProbabilisticSplits :163-224 for one file. */
int64_t or_probabilistic_splits(const uint8_t* f, uint64_t len, const uint64_t* beg,
                                const uint64_t* end, uint64_t n, uint64_t* v_start,
                                uint64_t* v_end) {
  /* BAMSplitGuesser(ss, conf): header read through SAMHeaderReader, magic check :85-87 */
  or_header h;
  int rc = or_read_header(f, len, &h);
  if (rc) return rc;
  return or_probabilistic_splits_nref(f, len, beg, end, n, h.n_ref, v_start, v_end);
}

/* the same over a window of the file whose header was read elsewhere (n_ref given) */
int64_t or_probabilistic_splits_nref(const uint8_t* f, uint64_t len, const uint64_t* beg,
                                     const uint64_t* end, uint64_t n, int32_t n_ref,
                                     uint64_t* v_start, uint64_t* v_end) {
  if (len < 4 || rd_i32(f) != BGZF_MAGIC) return OR_EFORMAT;
  guesser* g = guesser_new(f, len, n_ref);
  if (!g) return OR_ENOMEM;
  int64_t out = 0;
  for (uint64_t i = 0; i < n; ++i) {
    int err;
    const int64_t aligned_beg = g_guess(g, (int64_t)beg[i], (int64_t)end[i], &err);
    if (err) { out = err; break; }
    const uint64_t aligned_end = end[i] << 16 | 0xffff;
    if (aligned_beg == (int64_t)end[i]) {
      if (out == 0) { out = OR_EIO; break; } /* "no reads in first split" */
      v_end[out - 1] = aligned_end;
    } else {
      v_start[out] = (uint64_t)aligned_beg;
      v_end[out] = aligned_end;
      ++out;
    }
  }
  guesser_free(g);
  return out;
}

/* ------------------------------------------------------------------------------ */
/* SplittingBAMIndexer.index :146-186, skipToAlignmentList :188-223,
 * readAlignment :235-248, fullySkip :250-263 (stream BCIS, sequential). */
static int idx_read_bytes(bcis* b, uint8_t* buf, int32_t n, int32_t* got) {
  int32_t r = 0;
  while (r < n) {
    int32_t now;
    int rc = bcis_read(b, buf + r, n - r, &now);
    if (rc) return rc;
    if (now <= 0) break;
    r += now;
  }
  *got = r;
  return OR_OK;
}
static int idx_skip(bcis* b, int64_t s) {
  uint8_t tmp[2048];
  while (s > 0) {
    int32_t now;
    int rc = bcis_read(b, tmp, s > 2048 ? 2048 : (int32_t)s, &now);
    if (rc) return rc;
    if (now <= 0) return OR_EIO; /* "Skip failed" */
    s -= now;
  }
  return OR_OK;
}
int64_t or_splitting_index(const uint8_t* f, uint64_t len, int32_t granularity, uint64_t* out,
                           uint64_t cap) {
  ostream s = {f, (int64_t)len, 0};
  bcis* b = bcis_new(&s, 0);
  if (!b) return OR_ENOMEM;
  int64_t n = 0;
  int rc;
  int32_t got;
  uint8_t t[4];
  rc = idx_read_bytes(b, t, 4, &got);
  if (rc || got != 4 || memcmp(t, "BAM\1", 4) != 0) { n = rc ? rc : OR_EIO; goto out; }
  rc = idx_read_bytes(b, t, 4, &got);
  if (rc || got != 4) { n = rc ? rc : OR_EIO; goto out; }
  int32_t sam_len = rd_i32(t);
  if (sam_len < 0) { n = OR_EIO; goto out; }
  if ((rc = idx_skip(b, sam_len))) { n = rc; goto out; }
  rc = idx_read_bytes(b, t, 4, &got);
  if (rc || got != 4) { n = rc ? rc : OR_EIO; goto out; }
  int32_t nrefs = rd_i32(t);
  for (int32_t i = 0; i < nrefs; ++i) {
    rc = idx_read_bytes(b, t, 4, &got);
    if (rc || got != 4) { n = rc ? rc : OR_EIO; goto out; }
    if ((rc = idx_skip(b, (int64_t)rd_i32(t) + 4))) { n = rc; goto out; }
  }
  if ((uint64_t)n < cap) out[n] = bcis_tell(b);
  ++n;
  for (int32_t i = 0;;) {
    const uint64_t ptr = bcis_tell(b);
    rc = idx_read_bytes(b, t, 4, &got);
    if (rc) { n = rc; goto out; }
    if (got != 4) {
      if (got == 0) break;
      n = OR_EIO;
      goto out;
    }
    if (++i == granularity) {
      i = 0;
      if ((uint64_t)n < cap) out[n] = ptr;
      ++n;
    }
    if ((rc = idx_skip(b, rd_i32(t)))) { n = rc; goto out; }
  }
  if ((uint64_t)n < cap) out[n] = len << 16;
  ++n;
out:
  bcis_free(b);
  return n;
}

/* FileInputStream.read into dst: up to k bytes, 0 at or past EOF. */
static int bi_read(const uint8_t* f, uint64_t len, uint64_t* at, uint8_t* dst, int k) {
  if (*at >= len) return 0;
  const uint64_t avail = len - *at;
  const int got = avail < (uint64_t)k ? (int)avail : k;
  memcpy(dst, f + *at, (size_t)got);
  *at += (uint64_t)got;
  return got;
}

/* BGZFBlockIndexer.index + skipBlock (util/BGZFBlockIndexer.java:97-181) over a plain
 * FileInputStream: reads at or past EOF return 0 bytes; InputStream.skip on a file moves the
 * position by the full request even past EOF (so a truncated final block still counts).
 * Reference quirk kept: `pos` is a Java int (:88), so past 2 GiB it wraps and the entry is
 * the low 48 bits of the sign-extended value (lb.put(0, pos), :115-116).  Entries: `pos`
 * after every granularity-th block, then file.length() (:124-125).  Returns the count or
 * OR_EIO (the IOException ioError/"block without BGZF subfield" raise). */
int64_t or_bgzf_block_index(const uint8_t* f, uint64_t len, int32_t granularity, uint64_t* out,
                            uint64_t cap) {
  if (granularity <= 0) return OR_EIO;
  uint64_t at = 0;  /* FileInputStream position */
  int32_t pos = 0;  /* the indexer's int `pos` */
  int64_t n = 0;
  for (int32_t i = 0;;) {
    uint8_t bb[8];
    int got = bi_read(f, len, &at, bb, 4);
    if (got != 4) {
      if (got == 0) break;
      return OR_EIO; /* "too short, no ID/CM/FLG" */
    }
    if (((uint32_t)bb[0] << 24 | (uint32_t)bb[1] << 16 | (uint32_t)bb[2] << 8 | bb[3]) != 0x1f8b0804u)
      return OR_EIO;
    if (bi_read(f, len, &at, bb, 8) != 8) return OR_EIO; /* "no XLEN" */
    const int xlen = bb[6] | bb[7] << 8;
    int found = 0;
    for (int off = 0; off < xlen;) {
      if (bi_read(f, len, &at, bb, 4) != 4) return OR_EIO;
      off += 4;
      const uint32_t si = (uint32_t)bb[0] << 24 | (uint32_t)bb[1] << 16 | (uint32_t)bb[2] << 8 | bb[3];
      if ((si & ~0xffu) == 0x42430200u) {
        if (bi_read(f, len, &at, bb, 2) != 2) return OR_EIO; /* "missing BSIZE" */
        off += 2;
        const int bsize = bb[0] | bb[1] << 8;
        const int64_t skip = (int64_t)(xlen - off) + (bsize - xlen - 19) + 8;
        if (skip > 0) at += (uint64_t)skip; /* fullySkip: for (s = skip; s > 0;) */
        pos = (int32_t)((uint32_t)pos + (uint32_t)(bsize + 1));
        found = 1;
        break;
      }
      const int slen = bb[2] | bb[3] << 8;
      if (slen > 0) at += (uint64_t)slen;
      off += slen;
    }
    if (!found) return OR_EIO; /* "block without BGZF subfield" */
    if (++i == granularity) {
      i = 0;
      if ((uint64_t)n < cap) out[n] = (uint64_t)(int64_t)pos & 0xffffffffffffull;
      ++n;
    }
  }
  if ((uint64_t)n < cap) out[n] = len & 0xffffffffffffull;
  return n + 1;
}

/* ------------------------------------------------------------------------------ */
/* Columnar capture of the split reader (test/baseline helper).                      */
typedef struct cols_ctx {
  or_cols* c;
  int keep_var;
  int oom;
} cols_ctx;

#define GROW(field, type)                                                     \
  do {                                                                        \
    type* np = (type*)realloc(c->field, (size_t)ncap * sizeof(type));         \
    if (!np) return 1;                                                        \
    c->field = np;                                                            \
  } while (0)

static int cols_cb(void* user, const or_record* r) {
  cols_ctx* x = (cols_ctx*)user;
  or_cols* c = x->c;
  if (c->n + 1 >= c->cap) {
    uint64_t ncap = c->cap ? c->cap * 2 : 4096;
    GROW(voffset, uint64_t); GROW(key, int64_t); GROW(block_size, int32_t);
    GROW(ref_id, int32_t); GROW(pos, int32_t); GROW(l_read_name, uint8_t);
    GROW(mapq, uint8_t); GROW(bin, uint16_t); GROW(n_cigar, uint16_t); GROW(flag, uint16_t);
    GROW(l_seq, int32_t); GROW(next_ref_id, int32_t); GROW(next_pos, int32_t);
    GROW(tlen, int32_t); GROW(var_off, uint64_t);
    c->cap = ncap;
  }
  uint64_t i = c->n;
  if (i == 0) c->var_off[0] = 0;
  c->voffset[i] = r->voffset; c->key[i] = r->key; c->block_size[i] = r->block_size;
  c->ref_id[i] = r->ref_id; c->pos[i] = r->pos; c->l_read_name[i] = r->l_read_name;
  c->mapq[i] = r->mapq; c->bin[i] = r->bin; c->n_cigar[i] = r->n_cigar; c->flag[i] = r->flag;
  c->l_seq[i] = r->l_seq; c->next_ref_id[i] = r->next_ref_id; c->next_pos[i] = r->next_pos;
  c->tlen[i] = r->tlen;
  uint64_t vl = x->keep_var ? (uint64_t)(r->block_size - 32) : 0;
  uint64_t base = c->var_off[i];
  if (base + vl > c->var_cap) {
    uint64_t ncap = c->var_cap ? c->var_cap * 2 : (1u << 20);
    while (ncap < base + vl) ncap *= 2;
    uint8_t* np = (uint8_t*)realloc(c->var, ncap);
    if (!np) { x->oom = 1; return 1; }
    c->var = np;
    c->var_cap = ncap;
  }
  if (vl) memcpy(c->var + base, r->var, vl);
  c->var_off[i + 1] = base + vl;
  c->n = i + 1;
  return 0;
}
#undef GROW

int or_read_split_cols_nref(const uint8_t* f, uint64_t len, uint64_t v_start, uint64_t v_end,
                            int check_crc, int keep_var, int32_t n_ref, or_cols* out) {
  memset(out, 0, sizeof *out);
  cols_ctx x = {out, keep_var, 0};
  or_read_result res;
  if (n_ref < 0)
    or_read_split(f, len, v_start, v_end, check_crc, cols_cb, &x, &res);
  else
    read_split_body(f, len, v_start, v_end, check_crc, n_ref, cols_cb, &x, &res);
  out->status = x.oom ? OR_ENOMEM : res.status;
  out->err_record = res.err_record;
  if (out->n == 0 && out->var_off == NULL) {
    out->var_off = (uint64_t*)calloc(1, sizeof(uint64_t));
  }
  return out->status;
}

int or_read_split_cols(const uint8_t* f, uint64_t len, uint64_t v_start, uint64_t v_end,
                       int check_crc, int keep_var, or_cols* out) {
  return or_read_split_cols_nref(f, len, v_start, v_end, check_crc, keep_var, -1, out);
}

void or_cols_free(or_cols* c) {
  free(c->voffset); free(c->key); free(c->block_size); free(c->ref_id); free(c->pos);
  free(c->l_read_name); free(c->mapq); free(c->bin); free(c->n_cigar); free(c->flag);
  free(c->l_seq); free(c->next_ref_id); free(c->next_pos); free(c->tlen); free(c->var_off);
  free(c->var);
  memset(c, 0, sizeof *c);
}

/* ------------------------------------------------------------------------------ */
/* CPU baseline with the device path's whole output (bench.py cpu_baseline): the columns of
 * or_read_split_cols plus the lazy getters' pools the device decode materialises (names, CIGAR
 * u32s, SEQ as "=ACMGRSVTWYHKDBN" characters, QUAL, AUX, as check_one below defines them), built
 * into growing host buffers per split.  Returns the status; *pool_bytes = the pools' total size. */
typedef struct pools_ctx {
  cols_ctx cx;
  uint8_t* p;  /* one arena for the five pools (names | cigars | seq | qual | aux per record) */
  uint64_t n, cap;
  uint64_t* off; /* 5 offsets per record */
  uint64_t ocap;
} pools_ctx;

static const char SEQ_ALPHA_B[] = "=ACMGRSVTWYHKDBN";

static int pools_cb(void* user, const or_record* r) {
  pools_ctx* x = (pools_ctx*)user;
  if (cols_cb(&x->cx, r)) return 1;
  const int64_t vlen = (int64_t)r->block_size - 32;
  int64_t L = r->l_read_name, nc = r->n_cigar, ls = r->l_seq;
  const int64_t fixed = L + 4 * nc + (ls + 1) / 2 + ls;
  const int ok = ls >= 0 && fixed <= vlen;
  const int64_t na = ok ? vlen - fixed : 0;
  if (!ok) L = nc = ls = 0;
  const uint64_t need = (uint64_t)(L + 4 * nc + 2 * ls + na);
  if (x->n + need > x->cap) {
    uint64_t ncap = x->cap ? x->cap * 2 : (1u << 22);
    while (ncap < x->n + need) ncap *= 2;
    uint8_t* np = (uint8_t*)realloc(x->p, ncap);
    if (!np) { x->cx.oom = 1; return 1; }
    x->p = np;
    x->cap = ncap;
  }
  const uint64_t rec = x->cx.c->n - 1;
  if (5 * (rec + 1) > x->ocap) {
    uint64_t ncap = x->ocap ? x->ocap * 2 : 5 * 4096;
    uint64_t* np = (uint64_t*)realloc(x->off, ncap * sizeof(uint64_t));
    if (!np) { x->cx.oom = 1; return 1; }
    x->off = np;
    x->ocap = ncap;
  }
  const uint8_t* v = r->var;
  uint8_t* d = x->p + x->n;
  uint64_t* o = x->off + 5 * rec;
  o[0] = x->n;
  memcpy(d, v, (size_t)L);
  o[1] = x->n + (uint64_t)L;
  memcpy(d + L, v + L, (size_t)(4 * nc));
  const uint8_t* sp = v + L + 4 * nc;
  uint8_t* ds = d + L + 4 * nc;
  o[2] = x->n + (uint64_t)(L + 4 * nc);
  for (int64_t k = 0; k < ls; ++k) ds[k] = (uint8_t)SEQ_ALPHA_B[(k & 1) ? (sp[k >> 1] & 15) : (sp[k >> 1] >> 4)];
  const uint8_t* qp = sp + (ls + 1) / 2;
  o[3] = o[2] + (uint64_t)ls;
  memcpy(ds + ls, qp, (size_t)ls);
  o[4] = o[3] + (uint64_t)ls;
  memcpy(ds + 2 * ls, qp + ls, (size_t)na);
  x->n += need;
  return 0;
}

int or_read_split_pools(const uint8_t* f, uint64_t len, uint64_t v_start, uint64_t v_end, int32_t n_ref,
                        uint64_t* n_records, uint64_t* record_bytes, uint64_t* pool_bytes) {
  or_cols c;
  memset(&c, 0, sizeof c);
  pools_ctx x;
  memset(&x, 0, sizeof x);
  x.cx.c = &c;
  or_read_result res;
  if (n_ref < 0)
    or_read_split(f, len, v_start, v_end, 0, pools_cb, &x, &res);
  else
    read_split_body(f, len, v_start, v_end, 0, n_ref, pools_cb, &x, &res);
  uint64_t rb = 0;
  for (uint64_t i = 0; i < c.n; ++i) rb += (uint64_t)c.block_size[i] + 4u;
  *n_records = c.n;
  *record_bytes = rb;
  *pool_bytes = x.n;
  free(x.p);
  free(x.off);
  or_cols_free(&c);
  return x.cx.oom ? OR_ENOMEM : res.status;
}

/* ------------------------------------------------------------------------------ */
/* Whole-output checker (test infrastructure: bench.py's at-size parity).            */
enum {
  CK_COUNT = 1, CK_VOFFSET, CK_KEY, CK_FIXED, CK_BYTES, CK_LAYOUT, CK_NAMES, CK_CIGARS, CK_SEQ,
  CK_QUAL, CK_AUX
};

typedef struct check_ctx {
  const or_dev_cols* d;
  uint64_t next;  /* device index of the next oracle record */
  or_check* out;
} check_ctx;

static const char SEQ_ALPHA[] = "=ACMGRSVTWYHKDBN";

static int check_one(const or_dev_cols* d, uint64_t i, const or_record* r) {
  if (i >= d->n) return CK_COUNT;
  if (d->voffset[i] != r->voffset + d->voff_base) return CK_VOFFSET;
  if (d->key[i] != r->key) return CK_KEY;
  if (d->block_size[i] != r->block_size || d->ref_id[i] != r->ref_id || d->pos[i] != r->pos ||
      d->l_read_name[i] != r->l_read_name || d->mapq[i] != r->mapq || d->bin[i] != r->bin ||
      d->n_cigar[i] != r->n_cigar || d->flag[i] != r->flag || d->l_seq[i] != r->l_seq ||
      d->next_ref_id[i] != r->next_ref_id || d->next_pos[i] != r->next_pos || d->tlen[i] != r->tlen)
    return CK_FIXED;
  /* the record's bytes as the device holds them (rec_off: its block_size field) */
  const int64_t vlen = (int64_t)r->block_size - 32;
  if (d->rec_off[i] + 4u + (uint64_t)r->block_size > d->ubuf_len) return CK_BYTES;
  if (vlen > 0 && memcmp(d->ubuf + d->rec_off[i] + 36, r->var, (size_t)vlen) != 0) return CK_BYTES;
  /* lazy getters' pools (oracle.pools restated per record) */
  int64_t L = r->l_read_name, nc = r->n_cigar, ls = r->l_seq;
  const int64_t fixed = L + 4 * nc + (ls + 1) / 2 + ls;
  const int ok = ls >= 0 && fixed <= vlen;
  if (d->layout_ok[i] != (uint8_t)ok) return CK_LAYOUT;
  int64_t na = ok ? vlen - fixed : 0;
  if (!ok) L = nc = ls = 0;
  const uint8_t* v = r->var;
  if ((int64_t)(d->name_off[i + 1] - d->name_off[i]) != L ||
      (L && memcmp(d->names + d->name_off[i], v, (size_t)L) != 0))
    return CK_NAMES;
  if ((int64_t)(d->cigar_off[i + 1] - d->cigar_off[i]) != nc ||
      (nc && memcmp(d->cigars + d->cigar_off[i], v + L, (size_t)(4 * nc)) != 0))
    return CK_CIGARS;
  if ((int64_t)(d->seq_off[i + 1] - d->seq_off[i]) != ls) return CK_SEQ;
  const uint8_t* sp = v + L + 4 * nc;
  const uint8_t* ds = d->seq + d->seq_off[i];
  for (int64_t k = 0; k < ls; ++k) {
    const uint8_t nib = (k & 1) ? (sp[k >> 1] & 15) : (sp[k >> 1] >> 4);
    if (ds[k] != (uint8_t)SEQ_ALPHA[nib]) return CK_SEQ;
  }
  const uint8_t* qp = sp + (ls + 1) / 2;
  if (ls && memcmp(d->qual + d->seq_off[i], qp, (size_t)ls) != 0) return CK_QUAL;
  if ((int64_t)(d->aux_off[i + 1] - d->aux_off[i]) != na ||
      (na && memcmp(d->aux + d->aux_off[i], qp + ls, (size_t)na) != 0))
    return CK_AUX;
  return 0;
}

static int check_cb(void* user, const or_record* r) {
  check_ctx* x = (check_ctx*)user;
  const uint64_t i = x->next++;
  const int f = check_one(x->d, i, r);
  ++x->out->n_checked;
  if (f) {
    if (x->out->first_bad < 0) {
      x->out->first_bad = (int64_t)i;
      x->out->bad_field = f;
    }
    ++x->out->mismatches;
    if (f == CK_COUNT) return 1;  /* past the device's records: nothing more to compare */
  }
  return 0;
}

int or_check_split(const uint8_t* f, uint64_t len, uint64_t v_start, uint64_t v_end, int32_t n_ref,
                   const or_dev_cols* dev, uint64_t first, or_check* out) {
  memset(out, 0, sizeof *out);
  out->first_bad = -1;
  check_ctx x = {dev, first, out};
  or_read_result res;
  if (n_ref < 0)
    or_read_split(f, len, v_start, v_end, 0, check_cb, &x, &res);
  else
    read_split_body(f, len, v_start, v_end, 0, n_ref, check_cb, &x, &res);
  out->status = res.status;
  return res.status;
}

/* BCF read path: shares the stream model above */
#include "hbam_oracle_bcf.c"
