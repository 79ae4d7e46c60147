/* hbam_oracle_bcf.c — CPU restatement of Hadoop-BAM's BCF read path (TEST INFRASTRUCTURE).
 *
 * Compiled as part of hbam_oracle.c (included at its end: it reuses that file's ostream /
 * BlockCompressedInputStream model).  Restates
 *   - BCFSplitGuesser.guessNextBCFRecordStart / guessNextBGZFPos / guessNextBCFPos
 *     (BCFSplitGuesser.java:128-455), compressed and uncompressed;
 *   - BCFRecordReader.initialize / nextKeyValue (BCFRecordReader.java:71-174) with
 *     BGZFLimitingStream (:177-237);
 *   - [htsjdk] tribble PositionalBufferedStream (512,000-byte fills) and the parts of
 *     BCF2Codec.decode that decide whether bytes decode as a record (below).
 *
 * Parity: the candidate scan and the stream plumbing are the reference's own code.  The record
 * decode is htsjdk's BCF2Codec (absent: empty submodule), restated from the BCF2 spec as a
 * SUBSET — parity unpinned:
 *   1. l_shared, l_indiv: int32 read byte by byte (a byte past the end reads as 0xFF);
 *      negative -> TribbleException ("Invalid block size"); the site bytes must be readable
 *      (else TribbleException "Failed to read next complete record");
 *   2. site block (bytes past l_shared read as 0xFF, as the decoder's ByteArrayInputStream):
 *      CHROM int32 must index the contig dictionary (else IndexOutOfBoundsException, which
 *      escapes every catch of the reference); n_fmt_sample & 0xFFFFF must equal the header's
 *      sample count (TribbleException); n_allele >= 1 and n_fmt >= 0 (SitesInfoForDecoding
 *      .isValid, TribbleException);
 *   3. typed values ID, n_allele alleles, FILTER, n_info (key, value) must lie inside the site
 *      block (TribbleException; the decoder itself would read 0xFF past it); a descriptor whose
 *      type nibble is not 1/2/3/5/7 with a non-zero count escapes (no BCF2Type: NPE); an
 *      allele that is not a character string escapes (ClassCastException); FILTER and INFO
 *      key integers must index the string dictionary (IndexOutOfBoundsException escapes);
 *   4. the genotype bytes must be readable (TribbleException).
 * Allele-base validation and VariantContext.validate are not restated.
 */

#define BCF_PBS_SIZE 512000
#define BCF_UNCOMPRESSED_BYTES_NEEDED 0x80000
#define BCF_BGZF_BLOCKS_NEEDED 2
#define BCF_BGZF_MAX_BYTES_READ (BCF_BGZF_BLOCKS_NEEDED * 0xffff + 0xfffe)
#define BCF_SHORTEST_RECORD (4 * 8 + 1)

/* ---- InputStream sources under a PositionalBufferedStream ------------------------------- */
typedef struct bcf_src {
  int kind;        /* 0 ostream (uncompressed), 1 bcis, 2 BGZFLimitingStream over bcis */
  ostream* os;
  bcis* bz;
  uint64_t virt_end;
} bcf_src;

/* InputStream.read(byte[], 0, len): *got = bytes or -1; returns 0 or an error code */
static int src_read(bcf_src* s, uint8_t* buf, int32_t len, int32_t* got) {
  if (s->kind == 0) {
    *got = os_read(s->os, buf, len);
    return OR_OK;
  }
  if (s->kind == 1) return bcis_read(s->bz, buf, len, got);
  /* BGZFLimitingStream.read (BCFRecordReader.java:199-236) */
  int32_t total = 0, off = 0;
  uint64_t virt;
  const int32_t last_len = (int32_t)(s->virt_end & 0xffff);
  while (((virt = bcis_tell(s->bz)) >> 16) != (s->virt_end >> 16)) {
    int32_t r;
    const int32_t want = len < last_len ? len : last_len;
    if (want <= 0) return OR_EIO; /* read(buf, off, 0) forever: the reference would spin */
    int rc = bcis_read(s->bz, buf + off, want, &r);
    if (rc) return rc;
    if (r == -1) { *got = total == 0 ? -1 : total; return OR_OK; }
    total += r;
    len -= r;
    if (len == 0) { *got = total; return OR_OK; }
    off += r;
  }
  {
    const int32_t lim = (int32_t)(virt & 0xffff) - last_len;
    if (lim < len) len = lim;
  }
  while (len > 0) {
    int32_t r;
    int rc = bcis_read(s->bz, buf + off, len, &r);
    if (rc) return rc;
    if (r == -1) { *got = total == 0 ? -1 : total; return OR_OK; }
    total += r;
    len -= r;
    off += r;
  }
  *got = total == 0 ? -1 : total;
  return OR_OK;
}

/* ---- [htsjdk] tribble PositionalBufferedStream ----------------------------------------- */
typedef struct pbs {
  bcf_src* src;
  uint8_t* buf;
  int32_t n_chars, next;
  int64_t position;
} pbs;

static int pbs_init(pbs* p, bcf_src* s) {
  p->src = s;
  p->buf = (uint8_t*)malloc(BCF_PBS_SIZE);
  p->n_chars = p->next = 0;
  p->position = 0;
  return p->buf ? OR_OK : OR_ENOMEM;
}
static void pbs_free(pbs* p) { free(p->buf); p->buf = NULL; }
static int pbs_fill(pbs* p) {
  int32_t got;
  int rc = src_read(p->src, p->buf, BCF_PBS_SIZE, &got);
  if (rc) return rc;
  p->n_chars = got;
  p->next = 0;
  return OR_OK;
}
/* peek(): *c = next byte or -1 */
static int pbs_peek(pbs* p, int32_t* c) {
  for (;;) {
    if (p->n_chars < 0) { *c = -1; return OR_OK; }
    if (p->next == p->n_chars) {
      int rc = pbs_fill(p);
      if (rc) return rc;
      continue;
    }
    *c = p->buf[p->next];
    return OR_OK;
  }
}
static int pbs_read1(pbs* p, int32_t* c) {
  int rc = pbs_peek(p, c);
  if (rc) return rc;
  if (*c >= 0) { p->position++; p->next++; }
  return OR_OK;
}
/* read(bytes, 0, len): *got = bytes or -1 (isDone first) */
static int pbs_read(pbs* p, uint8_t* out, int32_t len, int32_t* got) {
  if (len == 0) { *got = 0; return OR_OK; }
  int32_t c;
  int rc = pbs_peek(p, &c); /* isDone() */
  if (rc) return rc;
  if (c < 0) { *got = -1; return OR_OK; }
  int32_t n = 0;
  while (len - n > 0) {
    if (p->n_chars == p->next) {
      rc = pbs_fill(p);
      if (rc) return rc;
      if (p->n_chars < 0) break;
    }
    int32_t k = p->n_chars - p->next;
    if (k > len - n) k = len - n;
    if (out) memcpy(out + n, p->buf + p->next, (size_t)k);
    p->next += k;
    n += k;
  }
  p->position += n;
  *got = n;
  return OR_OK;
}

/* ---- BCF2 record decode (restated subset, see the file header) -------------------------- */
typedef struct bcf_rec {
  int32_t l_shared, l_indiv, chrom, pos, rlen, n_allele, n_info, n_fmt, n_sample;
  uint32_t qual;     /* QUAL float bits */
  int32_t nai, nfs;  /* n_allele << 16 | n_info, n_fmt << 24 | n_sample as read */
  uint8_t* indiv;    /* the genotype block, when the caller asked for it (bcf_decode_keep) */
} bcf_rec;

typedef struct bcf_bytes { /* the decoder's ByteArrayInputStream over one block */
  const uint8_t* a;
  int32_t n, at;
} bcf_bytes;
static int32_t bb_byte(bcf_bytes* b) { return b->at < b->n ? b->a[b->at++] : (b->at++, 0xff); }
static int32_t bb_int(bcf_bytes* b, int nbytes) {
  uint32_t v = 0;
  for (int i = 0; i < nbytes; ++i) v |= (uint32_t)bb_byte(b) << (8 * i);
  if (nbytes == 1) return (int8_t)v;
  if (nbytes == 2) return (int16_t)v;
  return (int32_t)v;
}
static int type_bytes(int t) { return t == 1 ? 1 : t == 2 ? 2 : t == 3 ? 4 : t == 5 ? 4 : t == 7 ? 1 : 0; }
/* One typed value (descriptor, optional typed count, elements).  Restated rule: the value must
 * lie inside the site block (TribbleException otherwise); a non-empty value of a type nibble
 * other than 1/2/3/5/7 escapes (OR_ERUNTIME).  dict >= 0: the elements are dictionary offsets
 * (integers in [0, dict), else OR_ERUNTIME). */
static int bb_typed(bcf_bytes* b, int32_t dict, int* type, int32_t* count) {
  if (b->at >= b->n) return OR_ETRIBBLE;
  const int32_t d = b->a[b->at++];
  const int t = d & 0x0f;
  int64_t n = (d >> 4) & 0x0f;
  if (n == 15) { /* decodeNumberOfElements: a typed integer follows */
    if (b->at >= b->n) return OR_ETRIBBLE;
    const int t2 = b->a[b->at++] & 0x0f;
    if (!(t2 == 1 || t2 == 2 || t2 == 3)) return OR_ERUNTIME;
    if (b->at + type_bytes(t2) > b->n) return OR_ETRIBBLE;
    n = bb_int(b, type_bytes(t2));
  }
  *type = t;
  *count = (int32_t)n;
  if (n <= 0) return OR_OK; /* size 0: null, the type is never consulted */
  const int tb = type_bytes(t);
  if (!tb) return OR_ERUNTIME;
  if ((int64_t)b->at + n * tb > (int64_t)b->n) return OR_ETRIBBLE;
  if (dict >= 0) {
    if (!(t == 1 || t == 2 || t == 3)) return OR_ERUNTIME; /* (Integer) of a non-integer */
    for (int64_t i = 0; i < n; ++i) {
      const int32_t v = bb_int(b, tb);
      if (v < 0 || v >= dict) return OR_ERUNTIME;
    }
  } else {
    b->at += (int32_t)(n * tb);
  }
  return OR_OK;
}

typedef struct or_bcf_hdr_s {
  int32_t n_contig, n_sample, n_dict;
} or_bcf_hdr_s;

/* BCF2Codec.decode(PositionalBufferedStream), restated subset.  Returns 1 (a record), or an
 * error: OR_ETRIBBLE, OR_ERUNTIME, or a stream error of the fill (OR_EIO, OR_ETRUNC, ...). */
static int bcf_decode(pbs* p, const or_bcf_hdr_s* h, bcf_rec* r, uint8_t** scratch, int32_t* cap) {
  int32_t sz[2];
  for (int k = 0; k < 2; ++k) { /* BCF2Type.INT32.read: four read() calls, -1 & 0xFF */
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      int32_t c;
      int rc = pbs_read1(p, &c);
      if (rc) return rc;
      v |= (uint32_t)(c & 0xff) << (8 * i);
    }
    sz[k] = (int32_t)v;
  }
  r->l_shared = sz[0];
  r->l_indiv = sz[1];
  if (sz[0] < 0) return OR_ETRIBBLE;
  if (sz[0] > *cap) {
    uint8_t* q = (uint8_t*)realloc(*scratch, (size_t)sz[0] + 1);
    if (!q) return OR_ENOMEM;
    *scratch = q;
    *cap = sz[0];
  }
  { /* readRecordBytes: loop of read() calls, -1 -> TribbleException */
    int32_t n = 0;
    while (n < sz[0]) {
      int32_t got;
      int rc = pbs_read(p, *scratch + n, sz[0] - n, &got);
      if (rc) return rc;
      if (got < 0) return OR_ETRIBBLE;
      n += got;
    }
  }
  bcf_bytes b = {*scratch, sz[0], 0};
  r->chrom = bb_int(&b, 4);
  if (r->chrom < 0 || r->chrom >= h->n_contig) return OR_ERUNTIME; /* contigNames.get */
  r->pos = bb_int(&b, 4);
  r->rlen = bb_int(&b, 4);
  r->qual = (uint32_t)bb_int(&b, 4); /* QUAL */
  const int32_t nai = bb_int(&b, 4), nfs = bb_int(&b, 4);
  r->nai = nai;
  r->nfs = nfs;
  r->n_allele = nai >> 16;
  r->n_info = nai & 0xffff;
  r->n_fmt = nfs >> 24;
  r->n_sample = nfs & 0xfffff;
  if (r->n_sample != h->n_sample) return OR_ETRIBBLE;
  int t;
  int32_t cnt;
  int rc = bb_typed(&b, -1, &t, &cnt); /* ID */
  if (rc) return rc;
  for (int32_t i = 0; i < r->n_allele; ++i) { /* alleles: (String) decodeTypedValue() */
    rc = bb_typed(&b, -1, &t, &cnt);
    if (rc) return rc;
    if (cnt > 0 && t != 7) return OR_ERUNTIME;
  }
  rc = bb_typed(&b, h->n_dict, &t, &cnt); /* FILTER */
  if (rc) return rc;
  for (int32_t i = 0; i < r->n_info; ++i) {
    rc = bb_typed(&b, h->n_dict, &t, &cnt); /* key */
    if (rc) return rc;
    rc = bb_typed(&b, -1, &t, &cnt); /* value */
    if (rc) return rc;
  }
  if (r->n_fmt < 0 || r->n_allele < 1) return OR_ETRIBBLE; /* SitesInfoForDecoding.isValid */
  if (sz[1] < 0) return OR_ETRIBBLE;
  { /* genotype block: read and dropped (decoded lazily); kept in r->indiv when asked */
    int32_t n = 0;
    uint8_t* keep = NULL;
    if (r->indiv) {
      keep = (uint8_t*)realloc(r->indiv, (size_t)sz[1] + 1);
      if (!keep) return OR_ENOMEM;
      r->indiv = keep;
    }
    while (n < sz[1]) {
      int32_t got;
      rc = pbs_read(p, keep ? keep + n : NULL, sz[1] - n, &got);
      if (rc) return rc;
      if (got < 0) return OR_ETRIBBLE;
      n += got;
    }
  }
  return 1;
}

/* ---- header --------------------------------------------------------------------------- */
static int bcf_starts_with(const char* s, const char* e, const char* pfx) {
  size_t n = strlen(pfx);
  return (size_t)(e - s) >= n && memcmp(s, pfx, n) == 0;
}
/* BCF2Codec.readHeader (magic "BCF" 2.x, l_text, VCF text): contig lines, samples and the
 * string dictionary (BCF2Utils.makeDictionary: PASS, then FILTER / INFO / FORMAT IDs in header
 * order, first occurrence).  u: uncompressed stream bytes.  Returns OR_OK, OR_EEOF (need more
 * bytes) or OR_ETRIBBLE. */
int or_bcf_read_header(const uint8_t* u, uint64_t n, int32_t* n_contig, int32_t* n_sample,
                       int32_t* n_dict, uint64_t* header_len) {
  if (n < 9) return OR_EEOF;
  if (!(u[0] == 'B' && u[1] == 'C' && u[2] == 'F' && u[3] == 2 && u[4] >= 1)) return OR_ETRIBBLE;
  const int32_t lt = rd_i32(u + 5);
  if (lt <= 0) return OR_ETRIBBLE;
  if ((uint64_t)lt + 9 > n) return OR_EEOF;
  const char* t = (const char*)u + 9;
  const char* te = t + lt;
  int32_t nc = 0, ns = 0, nd = 1; /* PASS */
  /* IDs already in the dictionary (linear scan: headers are small) */
  const char* ids[4096];
  int32_t idl[4096];
  int32_t nid = 0;
  for (const char* l = t; l < te;) {
    const char* le = memchr(l, '\n', (size_t)(te - l));
    if (!le) le = te;
    if (bcf_starts_with(l, le, "##contig=<")) {
      ++nc;
    } else if (bcf_starts_with(l, le, "##FILTER=<") || bcf_starts_with(l, le, "##INFO=<") ||
               bcf_starts_with(l, le, "##FORMAT=<")) {
      const char* id = NULL;
      for (const char* q = l; q + 3 < le; ++q)
        if ((q[-1] == '<' || q[-1] == ',') && memcmp(q, "ID=", 3) == 0) { id = q + 3; break; }
      if (id) {
        const char* ie = id;
        while (ie < le && *ie != ',' && *ie != '>') ++ie;
        int seen = (ie - id == 4 && memcmp(id, "PASS", 4) == 0);
        for (int32_t k = 0; k < nid && !seen; ++k)
          seen = idl[k] == (int32_t)(ie - id) && memcmp(ids[k], id, (size_t)(ie - id)) == 0;
        if (!seen && nid < 4096) {
          ids[nid] = id;
          idl[nid++] = (int32_t)(ie - id);
          ++nd;
        }
      }
    } else if (bcf_starts_with(l, le, "#CHROM")) {
      int32_t cols = 1;
      for (const char* q = l; q < le; ++q) cols += *q == '\t';
      ns = cols > 9 ? cols - 9 : 0;
    }
    l = le + 1;
  }
  if (nc == 0) return OR_ETRIBBLE; /* "Didn't find any contig lines in BCF2 file header" */
  *n_contig = nc;
  *n_sample = ns;
  *n_dict = nd;
  *header_len = (uint64_t)lt + 9;
  return OR_OK;
}

/* ---- BCFSplitGuesser ---------------------------------------------------------------------- */
/* guessNextBCFPos :370-455 over cin (bcis for BGZF, the window stream otherwise) */
/* The method catches IOException only (:453): a FileTruncatedException or SAMFormatException
 * from a read that runs into the next block (the last reads reach 4 bytes past csize) escapes
 * (*esc). */
static int32_t g_next_bcf(guesser* g, bcf_src* cin, uint64_t cpv, int32_t up, int32_t csize,
                          const or_bcf_hdr_s* h, int* esc) {
  int32_t got;
  int rc_;
#define CSEEK(v)                                                              \
  do {                                                                        \
    if (cin->kind == 0) { if (os_seek(cin->os, (int64_t)(v))) return -1; }   \
    else if ((rc_ = bcis_seek(cin->bz, (v)))) { if (rc_ != OR_EIO) *esc = rc_; return -1; } \
  } while (0)
#define CREAD(n)                                                              \
  do {                                                                        \
    if (cin->kind == 0) got = os_read(cin->os, g->buf, (n));                  \
    else if ((rc_ = bcis_read(cin->bz, g->buf, (n), &got))) { if (rc_ != OR_EIO) *esc = rc_; return -1; } \
  } while (0)
  for (; up + BCF_SHORTEST_RECORD < csize; ++up) {
    CSEEK(cpv | (uint64_t)(int64_t)up);
    CREAD(8);
    const int64_t shared = (int64_t)(uint32_t)g_buf_i32(g, 0), indiv = (int64_t)(uint32_t)g_buf_i32(g, 4);
    if (shared + indiv < (int64_t)BCF_SHORTEST_RECORD) continue;
    CSEEK(cpv | (uint64_t)(int64_t)(up + 8));
    CREAD(8);
    const int32_t chrom = g_buf_i32(g, 0), pos = g_buf_i32(g, 4);
    if (chrom < 0 || chrom >= h->n_contig || pos < 0) continue;
    CSEEK(cpv | (uint64_t)(int64_t)(up + 24));
    CREAD(4);
    const int32_t ai = g_buf_i32(g, 0);
    const int32_t n_allele = ai >> 16, n_info = ai & 0xffff;
    if (n_allele < 0 || n_info < 0) continue;
    CSEEK(cpv | (uint64_t)(int64_t)(up + 28));
    CREAD(1);
    if ((int32_t)g->buf[0] != h->n_sample) continue;
    CSEEK(cpv | (uint64_t)(int64_t)(up + 32));
    CREAD(6);
    const int8_t id_type = (int8_t)g->buf[0];
    if ((id_type & 0x0f) != 0x07) continue;
    if ((id_type & 0xf0) == 0xf0) {
      const int8_t lt = (int8_t)g->buf[1];
      int64_t id_len;
      switch (lt & 0x0f) {
        case 1: id_len = g->buf[2]; break;
        case 2: id_len = g_ushort(g, 2); break;
        case 3: id_len = (int64_t)(uint32_t)g_buf_i32(g, 2); break;
        default: continue;
      }
      if (id_len < 15 || id_len > shared - (4 * 8 + n_allele + (int64_t)n_info * 2)) continue;
    }
    return up;
  }
#undef CSEEK
#undef CREAD
  return -1;
}

/* guessNextBCFRecordStart :128-281.  *err: OR_OK, or the exception that escapes the method. */
static int64_t g_guess_bcf(guesser* g, int64_t beg, int64_t end, int is_bgzf, const or_bcf_hdr_s* h,
                           int* err) {
  *err = OR_OK;
  const int32_t cap = is_bgzf ? BCF_BGZF_MAX_BYTES_READ : BCF_UNCOMPRESSED_BYTES_NEEDED;
  int32_t want = (int32_t)(end - beg);
  if (want > cap) want = cap;
  int64_t total = 0;
  if (want > 0 && beg >= 0 && beg <= g->flen) total = g->flen - beg < want ? g->flen - beg : want;
  g->in.a = g->file + (beg >= 0 && beg <= g->flen ? beg : 0);
  g->in.len = total;
  g->in.pos = 0;
  bcis_free(g->bgzf);
  g->bgzf = NULL;
  bcf_src cin = {0, &g->in, NULL, 0};
  int32_t first_end = 0;
  if (is_bgzf) {
    g->bgzf = bcis_new(&g->in, 1);
    if (!g->bgzf) { *err = OR_ENOMEM; return end; }
    cin.kind = 1;
    cin.bz = g->bgzf;
    first_end = (int32_t)(end - beg) < 0xffff ? (int32_t)(end - beg) : 0xffff;
  }
  uint8_t* scratch = NULL;
  int32_t scap = 0;
  int64_t result = end;
  for (int32_t cp = 0;; ++cp) {
    int32_t cp0;
    uint64_t cp0v;
    int32_t block_len;
    if (is_bgzf) {
      int32_t psz_pos, psz_size;
      if (!g_next_bgzf(g, cp, first_end, &psz_pos, &psz_size)) break;
      cp0 = cp = psz_pos;
      cp0v = (uint64_t)(uint32_t)cp0 << 16;
      if (bcis_seek(g->bgzf, cp0v)) continue; /* catch (Throwable) */
      block_len = psz_size;
    } else {
      cp0 = 0;
      cp0v = 0;
      block_len = (int32_t)total > BCF_UNCOMPRESSED_BYTES_NEEDED ? (int32_t)total : BCF_UNCOMPRESSED_BYTES_NEEDED;
    }
    for (int32_t up = 0;; ++up) {
      int esc = OR_OK;
      const int32_t up0 = up = g_next_bcf(g, &cin, cp0v, up, block_len, h, &esc);
      if (esc) { *err = esc; goto out; }
      if (up0 < 0) break;
      if (is_bgzf) {
        if (bcis_seek(g->bgzf, cp0v | (uint32_t)up0)) { *err = OR_EIO; goto out; }
      } else if (os_seek(&g->in, up0)) {
        *err = OR_EIO;
        goto out;
      }
      pbs pb;
      if (pbs_init(&pb, &cin)) { *err = OR_ENOMEM; goto out; }
      int decoded_any = 0, rc = OR_OK;
      int32_t c;
      if (is_bgzf) {
        int b = 0;
        const int32_t prev_cp = cp0; /* never updated (:216-231) */
        for (;;) {
          if (b >= BCF_BGZF_BLOCKS_NEEDED) break;
          rc = pbs_peek(&pb, &c);
          if (rc) break;
          if (c == -1) break;
          bcf_rec r;
          r.indiv = NULL;
          rc = bcf_decode(&pb, h, &r, &scratch, &scap);
          if (rc != 1) break;
          rc = OR_OK;
          decoded_any = 1;
          const int32_t cp2 = (int32_t)(bcis_tell(g->bgzf) >> 16);
          if (cp2 != prev_cp) { cp = cp2; ++b; }
        }
        if (rc == OR_OK && b < BCF_BGZF_BLOCKS_NEEDED && !decoded_any) { pbs_free(&pb); continue; }
      } else {
        for (;;) {
          if (!(pb.position - up0 < BCF_UNCOMPRESSED_BYTES_NEEDED)) break;
          rc = pbs_peek(&pb, &c);
          if (rc) break;
          if (c == -1) break;
          bcf_rec r;
          r.indiv = NULL;
          rc = bcf_decode(&pb, h, &r, &scratch, &scap);
          if (rc != 1) break;
          rc = OR_OK;
          decoded_any = 1;
        }
        if (rc == OR_OK && pb.position - up0 < BCF_UNCOMPRESSED_BYTES_NEEDED && !decoded_any) {
          pbs_free(&pb);
          continue;
        }
      }
      if (rc != OR_OK) {
        /* catch clauses :258-273 */
        if (rc == OR_ETRUNC || rc == OR_ENOMEM || rc == OR_EEOF) { pbs_free(&pb); continue; }
        if (rc == OR_ETRIBBLE) {
          int32_t pc = 0;
          int prc = decoded_any ? pbs_peek(&pb, &pc) : OR_OK;
          if (prc) { pbs_free(&pb); *err = prc; goto out; } /* peek() inside the handler throws */
          if (!(decoded_any && pc == -1)) { pbs_free(&pb); continue; }
        } else {
          pbs_free(&pb);
          *err = rc; /* escapes guessNextBCFRecordStart */
          goto out;
        }
      }
      pbs_free(&pb);
      result = is_bgzf ? (int64_t)((uint64_t)(beg + cp0) << 16 | (uint32_t)up0) : beg + up0;
      goto out;
    }
    if (!is_bgzf) break;
  }
out:
  free(scratch);
  return result;
}

int64_t or_guess_bcf_record_start(const uint8_t* f, uint64_t len, int64_t beg, int64_t end, int is_bgzf,
                                  int32_t n_contig, int32_t n_sample, int32_t n_dict, int* err) {
  guesser* g = (guesser*)calloc(1, sizeof(guesser)); /* ByteBuffer.allocate(8): zeros */
  if (!g) { *err = OR_ENOMEM; return end; }
  g->file = f;
  g->flen = (int64_t)len;
  const or_bcf_hdr_s h = {n_contig, n_sample, n_dict};
  int64_t r = g_guess_bcf(g, beg, end, is_bgzf, &h, err);
  guesser_free(g);
  return r;
}

/* ---- BCFRecordReader --------------------------------------------------------------------- */
/* One split: BGZF (FileVirtualSplit [v_start, v_end)) or uncompressed (FileSplit [start,
 * start+length), start = v_start, length = v_end).  Per record: its stream position (voffset
 * for BGZF: getFilePointer() of the underlying BCIS is NOT the record's position once the PBS
 * has read ahead, so the position is reported in the PBS's own coordinate: bytes from the split
 * start), CHROM, POS, key = (long)chrom << 32 | (long)pos.  Returns the count; *status = the
 * exception nextKeyValue raised after them (0 = clean end). */
/* or_read_bcf_split plus every column BCFRecordReader's records carry (l_shared, l_indiv, rlen,
 * QUAL bits, n_allele_info, n_fmt_sample) and each record's bytes (l_shared, l_indiv, the site
 * block, the genotype block) concatenated into bytes[0, bytes_cap) at boff[i] (boff: cap + 1). */
int64_t or_read_bcf_split_ex(const uint8_t* f, uint64_t len, int is_bgzf, uint64_t v_start, uint64_t v_end,
                             int32_t n_contig, int32_t n_sample, int32_t n_dict, uint64_t header_len,
                             int64_t* rel, int32_t* chrom, int32_t* pos, int64_t* key, int32_t* l_shared,
                             int32_t* l_indiv, int32_t* rlen, uint32_t* qual, int32_t* nai, int32_t* nfs,
                             uint8_t* bytes, uint64_t bytes_cap, uint64_t* boff, uint64_t cap, int* status);
int64_t or_read_bcf_split(const uint8_t* f, uint64_t len, int is_bgzf, uint64_t v_start, uint64_t v_end,
                          int32_t n_contig, int32_t n_sample, int32_t n_dict, uint64_t header_len,
                          int64_t* rel, int32_t* chrom, int32_t* pos, int64_t* key, uint64_t cap,
                          int* status) {
  return or_read_bcf_split_ex(f, len, is_bgzf, v_start, v_end, n_contig, n_sample, n_dict, header_len, rel,
                              chrom, pos, key, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 0, NULL, cap, status);
}
int64_t or_read_bcf_split_ex(const uint8_t* f, uint64_t len, int is_bgzf, uint64_t v_start, uint64_t v_end,
                             int32_t n_contig, int32_t n_sample, int32_t n_dict, uint64_t header_len,
                             int64_t* rel, int32_t* chrom, int32_t* pos, int64_t* key, int32_t* l_shared,
                             int32_t* l_indiv, int32_t* rlen, uint32_t* qual, int32_t* nai, int32_t* nfs,
                             uint8_t* bytes, uint64_t bytes_cap, uint64_t* boff, uint64_t cap, int* status) {
  *status = OR_OK;
  const or_bcf_hdr_s h = {n_contig, n_sample, n_dict};
  ostream os = {f, (int64_t)len, 0};
  bcis* bz = NULL;
  bcf_src src = {0, &os, NULL, 0};
  int64_t limit = -1;
  pbs pb;
  int rc;
  if (is_bgzf) {
    bz = bcis_new(&os, 0);
    if (!bz) { *status = OR_ENOMEM; return 0; }
    rc = bcis_seek(bz, v_start);
    if (rc) { *status = rc; bcis_free(bz); return 0; }
    src.kind = 2;
    src.bz = bz;
    src.virt_end = v_end;
  } else {
    /* initContigDict reads the header through the PBS first, then skips to the split start */
    limit = (int64_t)(v_start + v_end);
  }
  if (pbs_init(&pb, &src)) { bcis_free(bz); *status = OR_ENOMEM; return 0; }
  if (!is_bgzf) {
    int32_t got;
    uint64_t skip = header_len;
    if ((rc = pbs_read(&pb, NULL, (int32_t)skip, &got))) { *status = rc; goto done0; }
    if ((int64_t)v_start > pb.position) {
      int64_t s = (int64_t)v_start - pb.position;
      while (s > 0) {
        const int32_t k = s > (1 << 30) ? (1 << 30) : (int32_t)s;
        if ((rc = pbs_read(&pb, NULL, k, &got))) { *status = rc; goto done0; }
        if (got < 0) break;
        s -= got;
      }
    }
  }
  {
    uint8_t* scratch = NULL;
    uint8_t* indiv = NULL;
    int32_t scap = 0;
    int64_t n = 0;
    uint64_t bo = 0;
    const int64_t base = pb.position;
    if (boff) boff[0] = 0;
    for (;;) {
      int32_t c;
      if ((rc = pbs_peek(&pb, &c))) { *status = rc; break; }
      if (c == -1) break;
      if (!is_bgzf && pb.position >= limit) break;
      const int64_t at = pb.position;
      bcf_rec r;
      r.indiv = NULL;
      r.indiv = bytes ? (indiv ? indiv : (uint8_t*)malloc(1)) : NULL;
      rc = bcf_decode(&pb, &h, &r, &scratch, &scap);
      if (bytes) indiv = r.indiv;
      if (rc != 1) { *status = rc; break; }
      if ((uint64_t)n < cap) {
        rel[n] = is_bgzf ? at - base : at;
        chrom[n] = r.chrom;
        pos[n] = r.pos;
        key[n] = (int64_t)((uint64_t)(int64_t)r.chrom << 32 | (uint64_t)(int64_t)r.pos);
        if (l_shared) {
          l_shared[n] = r.l_shared;
          l_indiv[n] = r.l_indiv;
          rlen[n] = r.rlen;
          qual[n] = r.qual;
          nai[n] = r.nai;
          nfs[n] = r.nfs;
        }
        if (bytes) {
          const uint64_t need = 8 + (uint64_t)r.l_shared + (uint64_t)r.l_indiv;
          if (bo + need <= bytes_cap) {
            memcpy(bytes + bo, &r.l_shared, 4);
            memcpy(bytes + bo + 4, &r.l_indiv, 4);
            memcpy(bytes + bo + 8, scratch, (size_t)r.l_shared);
            memcpy(bytes + bo + 8 + r.l_shared, indiv, (size_t)r.l_indiv);
          }
          bo += need;
          boff[n + 1] = bo;
        }
      }
      ++n;
    }
    free(scratch);
    free(indiv);
    pbs_free(&pb);
    bcis_free(bz);
    return n;
  }
done0:
  pbs_free(&pb);
  bcis_free(bz);
  return 0;
}
