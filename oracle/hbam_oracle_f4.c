/* hbam_oracle_f4.c — CPU restatement of the read-name / CIGAR keyed consumers (SURVEY.md §8
 * f-4).  TEST INFRASTRUCTURE ONLY (see hbam_oracle.h): tests/ use it as the checker of
 * libhbam.so's hbam_summarize_ranges / hbam_name_order / hbam_fixmate.
 *
 * Input everywhere: n BAM records as SAMRecordWritable payloads (block_size field + record,
 * SAMRecordWritable.java:62-63) at pay + off[i] — what a decoded split or a received shuffle
 * buffer holds.
 *
 * Parity status: the consumers' own logic (Summarize.java:693-755, FixMate.java:209-277,
 * BAMRecordReader.getKey0 :104-106) is restated line by line.  What they call in htsjdk 1.131
 * (absent here) is restated from its published behaviour and is PARITY UNPINNED:
 * SamPairUtil.setMateInfo / computeInsertSize, SAMRecord.computeIndexingBin, and
 * BAMRecordCodec.encode of a record whose attributes changed (BinaryTagCodec integer
 * re-typing, 4-bit sequence re-packing, absent-quality fill).  DESIGN.md §3 lists them.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "hbam_oracle.h"

static int32_t rd32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24);
}
static uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | p[1] << 8); }
static void wr32(uint8_t* p, int32_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)((uint32_t)v >> 8);
  p[2] = (uint8_t)((uint32_t)v >> 16);
  p[3] = (uint8_t)((uint32_t)v >> 24);
}
static void wr16(uint8_t* p, uint16_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
}

/* record field access on a payload (block_size at +0, fixed fields from +4) */
#define R_REF(r) rd32((r) + 4)
#define R_POS(r) rd32((r) + 8)
#define R_LRN(r) ((r)[12])
#define R_MAPQ(r) ((r)[13])
#define R_BIN(r) rd16((r) + 14)
#define R_NCIG(r) rd16((r) + 16)
#define R_FLAG(r) rd16((r) + 18)
#define R_LSEQ(r) rd32((r) + 20)
#define R_NREF(r) rd32((r) + 24)
#define R_NPOS(r) rd32((r) + 28)
#define R_TLEN(r) rd32((r) + 32)
#define R_VAR(r) ((r) + 36)

/* BAMRecordReader.getKey0 (BAMRecordReader.java:104-106): (long)refIdx << 32 | alignmentStart0,
 * the int sign-extended before the OR */
static int64_t get_key0(int32_t ref, int32_t start0) {
  return (int64_t)((uint64_t)(int64_t)ref << 32) | (int64_t)start0;
}

/* Record layout bounds (a decoded split hands out records whose variable fields overrun
 * block_size with status OK: htsjdk decodes those fields lazily and throws when one is read).
 * cigar_ok: name + CIGAR inside the record (getCigar's read); layout_ok: every field. */
static int cigar_ok(const uint8_t* r) {
  const int64_t bs = rd32(r);
  return bs >= 32 && 32 + (int64_t)R_LRN(r) + 4 * (int64_t)R_NCIG(r) <= bs;
}
static int layout_ok(const uint8_t* r) {
  const int64_t bs = rd32(r), ls = R_LSEQ(r);
  return bs >= 32 && ls >= 0 && 32 + (int64_t)R_LRN(r) + 4 * (int64_t)R_NCIG(r) + (ls + 1) / 2 + ls <= bs;
}

/* ---- Summarize (cli/plugins/chipster/Summarize.java:664-755) ---------------------------- */
/* Java int arithmetic (wraps) */
static int32_t iadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }

/* SummarizeRecordReader.nextKeyValue over the records of one split.  split_status: the
 * exception the base BAMRecordReader raises after the n records (OR_OK when none).  Returns
 * the ranges delivered; *status = the exception nextKeyValue raises after them:
 *   OR_EREFID (IllegalArgumentException) — CigarOperator.binaryToEnum of an op code > 8;
 *   -13 (IndexOutOfBoundsException) — a record whose CIGAR yields no range: ranges.get(0)
 *   at :715;
 *   OR_EFORMAT — the record's CIGAR lies outside its block_size (getCigar's lazy read throws
 *   a runtime exception in htsjdk; its class is parity unpinned).  cap too small -> -8. */
int64_t or_summarize_ranges(const uint8_t* pay, const uint64_t* off, uint64_t n, int32_t split_status,
                            int64_t* key, int32_t* beg, int32_t* end, uint8_t* rev, uint32_t* rec,
                            uint64_t cap, int32_t* status) {
  uint64_t k = 0;
  *status = split_status;
  for (uint64_t i = 0; i < n; ++i) {
    const uint8_t* r = pay + off[i];
    const uint16_t flag = R_FLAG(r);
    const int32_t ref = R_REF(r);
    const int32_t start = iadd(R_POS(r), 1); /* getAlignmentStart(), 1-based */
    /* :708-709 skip unmapped / unplaced records */
    if ((flag & 4u) || ref < 0 || start < 0) continue;
    if (!cigar_ok(r)) {
      *status = OR_EFORMAT;
      return (int64_t)k;
    }
    /* parseCIGAR (:719-755) */
    const uint8_t* cig = R_VAR(r) + R_LRN(r);
    const uint32_t nc = R_NCIG(r);
    const int rv = (flag & 0x10u) != 0;
    int32_t b = start, e = start;
    const uint64_t k0 = k;
    for (uint32_t j = 0; j < nc; ++j) {
      const uint32_t c = (uint32_t)rd32(cig + 4 * j);
      const uint32_t op = c & 15u;
      const int32_t len = (int32_t)(c >> 4);
      if (op > 8u) { /* BinaryCigarCodec -> CigarOperator.binaryToEnum */
        *status = OR_EREFID;
        return (int64_t)k0;
      }
      if (op == 0u || op == 7u || op == 8u) { /* M, =, X: accumulate */
        e = iadd(e, len);
        continue;
      }
      if (b != e) {
        if (k >= cap) return OR_ENOMEM;
        beg[k] = b;
        end[k] = iadd(e, -1);
        rev[k] = (uint8_t)rv;
        rec[k] = (uint32_t)i;
        ++k;
        b = e;
      }
      if (op == 2u || op == 3u) { /* D, N consume reference bases */
        b = iadd(b, len);
        e = b;
      }
    }
    if (b != e) {
      if (k >= cap) return OR_ENOMEM;
      beg[k] = b;
      end[k] = iadd(e, -1);
      rev[k] = (uint8_t)rv;
      rec[k] = (uint32_t)i;
      ++k;
    }
    if (k == k0) { /* ranges.get(0) on an empty list */
      *status = -13;
      return (int64_t)k0;
    }
    /* :714-715 first key; :696-699 each further range keeps the high word */
    for (uint64_t q = k0; q < k; ++q) {
      const int32_t com = (int32_t)(((int64_t)beg[q] + (int64_t)end[q]) / 2); /* getCentreOfMass */
      if (q == k0)
        key[q] = get_key0(ref, com);
      else
        key[q] = (int64_t)(((uint64_t)key[q - 1] >> 32) << 32) | (int64_t)com;
    }
  }
  return (int64_t)k;
}

/* ---- FixMate (cli/plugins/FixMate.java:209-277) --------------------------------------------- */
/* Map output key: Text(getReadName()).  getReadName = the l_read_name-1 name bytes; Text's
 * raw comparator is unsigned lexicographic with a proper prefix first, and the byte -> char ->
 * UTF-8 mapping htsjdk + Text apply is order preserving and prefix free, so comparing the raw
 * name bytes gives Text's order and Text's equality. */
static uint32_t name_len(const uint8_t* r) { return R_LRN(r) ? (uint32_t)R_LRN(r) - 1u : 0u; }
static int name_cmp(const uint8_t* a, const uint8_t* b) {
  const uint32_t la = name_len(a), lb = name_len(b);
  const int c = memcmp(R_VAR(a), R_VAR(b), la < lb ? la : lb);
  if (c) return c;
  return la < lb ? -1 : la > lb ? 1 : 0;
}

static const uint8_t* g_pay;
static const uint64_t* g_off;
static int perm_cmp(const void* x, const void* y) {
  const uint32_t i = *(const uint32_t*)x, j = *(const uint32_t*)y;
  const int c = name_cmp(g_pay + g_off[i], g_pay + g_off[j]);
  if (c) return c;
  return i < j ? -1 : i > j ? 1 : 0; /* documented tie-break: input order */
}

/* Shuffle order of FixMateMapper's output: records by (Text key, input order).  The reference's
 * order of equal keys is unspecified (spill QuickSort + merge); input order is the documented
 * choice, as for Sort. */
void or_name_order(const uint8_t* pay, const uint64_t* off, uint64_t n, uint32_t* perm) {
  for (uint64_t i = 0; i < n; ++i) perm[i] = (uint32_t)i;
  g_pay = pay;
  g_off = off;
  qsort(perm, n, sizeof(uint32_t), perm_cmp);
}

/* ---- htsjdk pieces the reducer calls (PARITY UNPINNED, see the header) -------------------- */
static int32_t ref_length(const uint8_t* r) { /* Cigar.getReferenceLength: M D N = X */
  const uint8_t* cig = R_VAR(r) + R_LRN(r);
  int32_t s = 0;
  for (uint32_t j = 0; j < R_NCIG(r); ++j) {
    const uint32_t c = (uint32_t)rd32(cig + 4 * j), op = c & 15u;
    if (op == 0u || op == 2u || op == 3u || op == 7u || op == 8u) s = iadd(s, (int32_t)(c >> 4));
  }
  return s;
}
/* GenomicIndexUtil.reg2bin(beg, end), end exclusive */
static int reg2bin(int beg, int end) {
  --end;
  if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
  if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
  if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
  if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
  if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
  return 0;
}

/* the mutable view of one record during the reducer (SAMRecord setters) */
typedef struct fm_rec {
  const uint8_t* r; /* original payload */
  int32_t ref, pos, nref, npos, tlen;
  uint16_t flag;
  int bin_stale;   /* setAlignmentStart cleared the indexing bin */
  int mq;          /* -1: leave MQ as it is, -2: remove, >= 0: set to this value */
  int drop_mc;     /* remove MC */
  int modified;    /* attributes touched: BAMRecordCodec re-serializes the record */
} fm_rec;

static void fm_load(fm_rec* f, const uint8_t* r) {
  f->r = r;
  f->ref = R_REF(r);
  f->pos = R_POS(r);
  f->nref = R_NREF(r);
  f->npos = R_NPOS(r);
  f->tlen = R_TLEN(r);
  f->flag = R_FLAG(r);
  f->bin_stale = 0;
  f->mq = -1;
  f->drop_mc = 0;
  f->modified = 0;
}
static int fm_unmapped(const fm_rec* f) { return (f->flag & 4u) != 0; }
static int fm_neg(const fm_rec* f) { return (f->flag & 0x10u) != 0; }
static int32_t fm_start(const fm_rec* f) { return iadd(f->pos, 1); }
static void fm_set_start(fm_rec* f, int32_t s) { /* setAlignmentStart: bin -> null */
  f->pos = iadd(s, -1);
  f->bin_stale = 1;
}
static void fm_mate_flags(fm_rec* f, int mate_neg, int mate_unmapped) {
  f->flag = (uint16_t)((f->flag & ~0x28u) | (mate_neg ? 0x20u : 0u) | (mate_unmapped ? 8u : 0u));
}
/* getAlignmentEnd: 0 for an unmapped read, else start + reference length - 1 */
static int32_t fm_end(const fm_rec* f) {
  if (fm_unmapped(f)) return 0;
  return iadd(iadd(fm_start(f), ref_length(f->r)), -1);
}
/* SamPairUtil.computeInsertSize(first, second) */
static int32_t insert_size(const fm_rec* a, const fm_rec* b) {
  if (fm_unmapped(a) || fm_unmapped(b)) return 0;
  if (a->ref != b->ref) return 0; /* getReferenceName().equals */
  const int32_t p1 = fm_neg(a) ? fm_end(a) : fm_start(a);
  const int32_t p2 = fm_neg(b) ? fm_end(b) : fm_start(b);
  return iadd(iadd(p2, -p1), p2 >= p1 ? 1 : -1);
}
/* SamPairUtil.setMateInfo(rec1, rec2, header) = setMateInfo(rec1, rec2, header, false) */
static void set_mate_info(fm_rec* a, fm_rec* b) {
  if (!fm_unmapped(a) && !fm_unmapped(b)) {
    a->nref = b->ref;
    a->npos = b->pos;
    fm_mate_flags(a, fm_neg(b), 0);
    a->mq = R_MAPQ(b->r);
    b->nref = a->ref;
    b->npos = a->pos;
    fm_mate_flags(b, fm_neg(a), 0);
    b->mq = R_MAPQ(a->r);
  } else if (fm_unmapped(a) && fm_unmapped(b)) {
    fm_rec* q[2] = {a, b};
    for (int t = 0; t < 2; ++t) {
      fm_rec* x = q[t];
      const fm_rec* y = q[1 - t];
      x->ref = -1;
      fm_set_start(x, 0);
      x->nref = -1;
      x->npos = -1; /* setMateAlignmentStart(0) */
      fm_mate_flags(x, fm_neg(y), 1);
      x->mq = -2;
      x->tlen = 0;
    }
  } else {
    fm_rec* m = fm_unmapped(a) ? b : a;
    fm_rec* u = fm_unmapped(a) ? a : b;
    u->ref = m->ref;
    fm_set_start(u, fm_start(m));
    m->nref = u->ref;
    m->npos = u->pos;
    fm_mate_flags(m, fm_neg(u), 1);
    m->mq = -2;
    m->tlen = 0;
    u->nref = m->ref;
    u->npos = m->pos;
    fm_mate_flags(u, fm_neg(m), 0);
    u->mq = R_MAPQ(m->r);
    u->tlen = 0;
  }
  a->drop_mc = b->drop_mc = 1;
  a->modified = b->modified = 1;
  const int32_t is = insert_size(a, b);
  a->tlen = is;
  b->tlen = iadd(0, -is);
}

/* BinaryTagCodec.getIntegerType */
static char int_type(int64_t v) {
  if (v > 2147483647LL) return 'I';
  if (v > 65535) return 'i';
  if (v > 255) return 'S';
  if (v > 127) return 'C';
  if (v >= -128) return 'c';
  if (v >= -32768) return 's';
  return 'i';
}
static uint32_t int_type_size(char t) { return t == 'c' || t == 'C' ? 1u : t == 's' || t == 'S' ? 2u : 4u; }
static void put_int(uint8_t* d, char t, int64_t v) {
  const uint32_t s = int_type_size(t);
  for (uint32_t k = 0; k < s; ++k) d[k] = (uint8_t)((uint64_t)v >> (8 * k));
}
/* size of one aux tag's value (after the 3-byte tag + type), or -1 when malformed */
static int64_t aux_value_size(const uint8_t* p, uint64_t avail, char t) {
  switch (t) {
    case 'A': case 'c': case 'C': return 1;
    case 's': case 'S': return 2;
    case 'i': case 'I': case 'f': return 4;
    case 'Z': case 'H': {
      for (uint64_t k = 0; k < avail; ++k)
        if (p[k] == 0) return (int64_t)k + 1;
      return -1;
    }
    case 'B': {
      if (avail < 5) return -1;
      const char st = (char)p[0];
      const uint32_t cnt = (uint32_t)rd32(p + 1);
      const uint32_t es = (st == 'c' || st == 'C') ? 1u : (st == 's' || st == 'S') ? 2u
                          : (st == 'i' || st == 'I' || st == 'f') ? 4u : 0u;
      if (!es) return -1;
      return 5 + (int64_t)cnt * es;
    }
    default: return -1;
  }
}
static int64_t aux_int(const uint8_t* p, char t) {
  switch (t) {
    case 'c': return (int8_t)p[0];
    case 'C': return p[0];
    case 's': return (int16_t)rd16(p);
    case 'S': return rd16(p);
    case 'i': return rd32(p);
    default: return (uint32_t)rd32(p);
  }
}

/* BAMRecordCodec.encode of the record (SAMRecordWritable.write).  An untouched record keeps
 * its bytes; a modified one is re-serialized: fixed fields from the setters (bin recomputed
 * after setAlignmentStart, 0 when refID < 0), the 4-bit sequence re-packed (odd length: zero
 * pad nibble), absent qualities (first byte 0xFF) written as 0xFF fill, every integer tag
 * re-typed by value, MC removed, MQ replaced in place / appended / removed.  Writes into dst
 * (NULL: size only).  Returns the payload length or -1 (malformed aux: SAMFormatException). */
static int64_t fm_encode(const fm_rec* f, uint8_t* dst) {
  const uint8_t* r = f->r;
  const int32_t bs = rd32(r);
  if (!f->modified) {
    if (dst) {
      memcpy(dst, r, (size_t)bs + 4);
      wr32(dst + 4, f->ref);
      wr32(dst + 8, f->pos);
      wr16(dst + 18, f->flag);
      wr32(dst + 24, f->nref);
      wr32(dst + 28, f->npos);
      wr32(dst + 32, f->tlen);
    }
    return (int64_t)bs + 4;
  }
  const uint32_t lrn = R_LRN(r), nc = R_NCIG(r);
  const int32_t lseq = R_LSEQ(r);
  const uint64_t ls = lseq > 0 ? (uint64_t)lseq : 0;
  const uint64_t head = 36 + lrn + 4ull * nc, sq = (ls + 1) / 2;
  const uint8_t* aux = r + head + sq + ls;
  const uint64_t aux_len = (uint64_t)bs + 4 - (head + sq + ls);
  uint64_t o = head + sq + ls;
  int mq_done = 0;
  /* aux walk */
  uint64_t p = 0;
  while (p < aux_len) {
    if (aux_len - p < 3) return -1;
    const uint8_t t0 = aux[p], t1 = aux[p + 1];
    const char ty = (char)aux[p + 2];
    const int64_t vs = aux_value_size(aux + p + 3, aux_len - p - 3, ty);
    if (vs < 0 || (uint64_t)vs > aux_len - p - 3) return -1;
    const int is_mc = t0 == 'M' && t1 == 'C', is_mq = t0 == 'M' && t1 == 'Q';
    if (is_mc && f->drop_mc) {
      /* removed */
    } else if (is_mq && f->mq != -1) {
      if (f->mq >= 0) {
        const char nt = int_type(f->mq);
        if (dst) {
          dst[o] = 'M';
          dst[o + 1] = 'Q';
          dst[o + 2] = (uint8_t)nt;
          put_int(dst + o + 3, nt, f->mq);
        }
        o += 3 + int_type_size(nt);
      }
      mq_done = 1;
    } else if (ty == 'c' || ty == 'C' || ty == 's' || ty == 'S' || ty == 'i' || ty == 'I') {
      const int64_t v = aux_int(aux + p + 3, ty);
      const char nt = int_type(v);
      if (dst) {
        dst[o] = t0;
        dst[o + 1] = t1;
        dst[o + 2] = (uint8_t)nt;
        put_int(dst + o + 3, nt, v);
      }
      o += 3 + int_type_size(nt);
    } else {
      if (dst) memcpy(dst + o, aux + p, 3 + (size_t)vs);
      o += 3 + (uint64_t)vs;
    }
    p += 3 + (uint64_t)vs;
  }
  if (!mq_done && f->mq >= 0) { /* appended at the end of the attribute list */
    const char nt = int_type(f->mq);
    if (dst) {
      dst[o] = 'M';
      dst[o + 1] = 'Q';
      dst[o + 2] = (uint8_t)nt;
      put_int(dst + o + 3, nt, f->mq);
    }
    o += 3 + int_type_size(nt);
  }
  if (dst) {
    memcpy(dst, r, head); /* block_size rewritten below */
    wr32(dst, (int32_t)(o - 4));
    wr32(dst + 4, f->ref);
    wr32(dst + 8, f->pos);
    uint16_t bin = R_BIN(r);
    if (f->ref < 0) {
      bin = 0;
    } else if (f->bin_stale) { /* SAMRecord.computeIndexingBin */
      const int32_t s0 = iadd(fm_start(f), -1);
      int32_t e = fm_end(f);
      if (e <= 0) e = iadd(s0, 1);
      bin = (uint16_t)reg2bin(s0, e);
    }
    wr16(dst + 14, bin);
    wr16(dst + 18, f->flag);
    wr32(dst + 24, f->nref);
    wr32(dst + 28, f->npos);
    wr32(dst + 32, f->tlen);
    memcpy(dst + head, r + head, sq);
    if (ls & 1u) dst[head + sq - 1] &= 0xf0u;
    if (ls && r[head + sq] == 0xffu)
      memset(dst + head + sq, 0xff, ls);
    else
      memcpy(dst + head + sq, r + head + sq, ls);
  }
  return (int64_t)o;
}

/* one reducer output: fm (copied) -> out */
static int fm_emit(const fm_rec* f, uint32_t src, uint8_t* out_pay, uint64_t* out_off, uint32_t* out_src,
                   uint64_t* k, uint64_t cap, uint64_t pay_cap) {
  const int64_t len = fm_encode(f, NULL);
  if (len < 0) return OR_EFORMAT;
  if (*k >= cap || out_off[*k] + (uint64_t)len > pay_cap) return OR_ENOMEM;
  fm_encode(f, out_pay + out_off[*k]);
  out_src[*k] = src;
  out_off[*k + 1] = out_off[*k] + (uint64_t)len;
  ++*k;
  return OR_OK;
}

/* FixMateReducer.reduce (FixMate.java:230-277) over every key group of the shuffle order
 * (or_name_order), without the combiner (FixMate -C).  Output: the reducer's writes in order,
 * each a SAMRecordWritable payload at out_pay + out_off[k] and the input record it came from.
 * Reproduced quirk: when a primary is followed only by secondaries, the inner loop ends with b
 * = the last secondary, which is then mated and written a second time.  Returns the output
 * count; *status = OR_EFORMAT when a touched record's attributes do not parse, or (no
 * outputs) when any record's fields overrun its block_size: the mapper's getReadName / lazy
 * field decode throws before the reducer runs. */
int64_t or_fixmate(const uint8_t* pay, const uint64_t* off, uint64_t n, uint8_t* out_pay, uint64_t* out_off,
                   uint32_t* out_src, uint64_t cap, uint64_t pay_cap, int32_t* status) {
  out_off[0] = 0;
  for (uint64_t i = 0; i < n; ++i)
    if (!layout_ok(pay + off[i])) {
      *status = OR_EFORMAT;
      return 0;
    }
  uint32_t* perm = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
  if (!perm) return OR_ENOMEM;
  or_name_order(pay, off, n, perm);
  uint64_t k = 0;
  out_off[0] = 0;
  *status = OR_OK;
  int rc = OR_OK;
  uint64_t g = 0;
  while (g < n && rc == OR_OK) {
    uint64_t ge = g + 1;
    while (ge < n && name_cmp(pay + off[perm[g]], pay + off[perm[ge]]) == 0) ++ge;
    uint64_t it = g; /* the values iterator */
    while (it < ge && rc == OR_OK) {
      fm_rec a;
      const uint32_t ai = perm[it++];
      fm_load(&a, pay + off[ai]);
      if (a.flag & 0x100u) { /* getNotPrimaryAlignmentFlag */
        rc = fm_emit(&a, ai, out_pay, out_off, out_src, &k, cap, pay_cap);
        continue;
      }
      fm_rec b;
      uint32_t bi = 0;
      int have_b = 0;
      while (it < ge && rc == OR_OK) {
        bi = perm[it++];
        fm_load(&b, pay + off[bi]);
        have_b = 1;
        if (!(b.flag & 0x100u)) break;
        rc = fm_emit(&b, bi, out_pay, out_off, out_src, &k, cap, pay_cap);
      }
      if (rc != OR_OK) break;
      if (!have_b) {
        rc = fm_emit(&a, ai, out_pay, out_off, out_src, &k, cap, pay_cap);
        break;
      }
      set_mate_info(&a, &b);
      rc = fm_emit(&a, ai, out_pay, out_off, out_src, &k, cap, pay_cap);
      if (rc == OR_OK) rc = fm_emit(&b, bi, out_pay, out_off, out_src, &k, cap, pay_cap);
    }
    g = ge;
  }
  free(perm);
  if (rc == OR_ENOMEM) return OR_ENOMEM;
  *status = rc;
  return (int64_t)k;
}
