// hbam_bcf.hip — BCF2 over the BGZF layer on the device, gfx950.
//
// The BCF read path reuses the BAM kernels unchanged below the record level: block framing
// (k_scan_chunks / k_verify_chain), the two-phase inflate (k_inflate_tokens + k_resolve), the
// guess window block cache, and the record-chain walk (k_block_entry / k_block_walk / stitch /
// repair, generic over the record format).  What differs is the record:
//   * BcfFmt — BCF2 framing for the chain walk: a record is l_shared u32 | l_indiv u32 |
//     site block | genotype block, next = r + 8 + l_shared + l_indiv; the per-block entry
//     predicate is BCFSplitGuesser.guessNextBCFPos' test (BCFSplitGuesser.java:370-455);
//   * bcf_site() — the restated subset of BCF2Codec.decode (parity unpinned; the same rules as
//     oracle/hbam_oracle_bcf.c, listed there);
//   * k_bcf_decode — BCFRecordReader.nextKeyValue (BCFRecordReader.java:158-174) per record:
//     status, CHROM/POS/rlen/QUAL/counts, key = (long)chrom << 32 | (long)pos;
//   * k_guess_bcf — BCFSplitGuesser.guessNextBCFRecordStart (:128-281), one lane per guess,
//     over the same window cache as the BAM guesser.  tribble's PositionalBufferedStream
//     (512,000-byte fills) is modelled without its buffer: a lead cursor performs each fill
//     (its exceptions, its end of stream, the getFilePointer() the verification loop reads) and
//     a trailing cursor over the same bytes yields the values the decode consumes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbam_internal.h"

namespace hbam {

constexpr int32_t BCF_PBS_SIZE = 512000;          // tribble PositionalBufferedStream buffer
constexpr int32_t BCF_UNCOMP_NEEDED = 0x80000;    // BCFSplitGuesser.java:64
constexpr int32_t BCF_BGZF_WINDOW = 2 * 0xffff + 0xfffe;  // :74-75
constexpr int32_t BCF_SHORTEST = 4 * 8 + 1;       // :82
constexpr int32_t BCF_MIN_SHARED = 27;  // fewer site bytes never decode (24 fixed + ID + allele + FILTER)

struct BcfHdr {
  int32_t n_contig, n_sample, n_dict;
};

// ---- the restated BCF2Codec site decode ---------------------------------------------------
// Sequential byte source over one site block of n bytes (bytes past n read as 0xFF, as the
// decoder's ByteArrayInputStream).  Src::at(i) for nondecreasing i.
struct BcfBytes {
  const uint8_t* a;
  __device__ __forceinline__ uint32_t at(int64_t i) { return a[i]; }
};
__device__ __forceinline__ int32_t bcf_tb(int t) {
  return t == 1 ? 1 : t == 2 ? 2 : t == 3 ? 4 : t == 5 ? 4 : t == 7 ? 1 : 0;
}
template <typename Src>
__device__ __forceinline__ int32_t bcf_rd(Src& s, int64_t n, int64_t& at, int nb) {
  uint32_t v = 0;
  for (int i = 0; i < nb; ++i, ++at) v |= (at < n ? s.at(at) : 0xffu) << (8 * i);
  return nb == 1 ? (int32_t)(int8_t)v : nb == 2 ? (int32_t)(int16_t)v : (int32_t)v;
}
// one typed value inside the block; dict >= 0: integer dictionary offsets
template <typename Src>
__device__ int32_t bcf_typed(Src& s, int64_t n, int64_t& at, int32_t dict, int* type, int64_t* count) {
  if (at >= n) return HBAM_ETRIBBLE;
  const uint32_t d = s.at(at++);
  const int t = (int)(d & 15u);
  int64_t k = (d >> 4) & 15u;
  if (k == 15) {
    if (at >= n) return HBAM_ETRIBBLE;
    const int t2 = (int)(s.at(at++) & 15u);
    if (!(t2 == 1 || t2 == 2 || t2 == 3)) return HBAM_ERUNTIME;
    if (at + bcf_tb(t2) > n) return HBAM_ETRIBBLE;
    k = bcf_rd(s, n, at, bcf_tb(t2));
  }
  *type = t;
  *count = k;
  if (k <= 0) return HBAM_OK;
  const int tb = bcf_tb(t);
  if (!tb) return HBAM_ERUNTIME;
  if (at + k * tb > n) return HBAM_ETRIBBLE;
  if (dict >= 0) {
    if (!(t == 1 || t == 2 || t == 3)) return HBAM_ERUNTIME;
    for (int64_t i = 0; i < k; ++i) {
      const int32_t v = bcf_rd(s, n, at, tb);
      if (v < 0 || v >= dict) return HBAM_ERUNTIME;
    }
  } else {
    at += k * tb;
  }
  return HBAM_OK;
}
struct BcfSite {
  int32_t chrom, pos, rlen, n_allele_info, n_fmt_sample;
  uint32_t qual;
};
// decodeSiteLoc + decodeSitesExtendedInfo over the site block (n = l_shared bytes):
// HBAM_OK, HBAM_ETRIBBLE or HBAM_ERUNTIME
template <typename Src>
__device__ int32_t bcf_site(Src& s, int64_t n, const BcfHdr& h, BcfSite* o) {
  int64_t at = 0;
  o->chrom = bcf_rd(s, n, at, 4);
  if (o->chrom < 0 || o->chrom >= h.n_contig) return HBAM_ERUNTIME;  // contigNames.get
  o->pos = bcf_rd(s, n, at, 4);
  o->rlen = bcf_rd(s, n, at, 4);
  o->qual = (uint32_t)bcf_rd(s, n, at, 4);
  o->n_allele_info = bcf_rd(s, n, at, 4);
  o->n_fmt_sample = bcf_rd(s, n, at, 4);
  const int32_t n_allele = o->n_allele_info >> 16, n_info = o->n_allele_info & 0xffff;
  if ((o->n_fmt_sample & 0xfffff) != h.n_sample) return HBAM_ETRIBBLE;
  int t;
  int64_t k;
  int32_t rc = bcf_typed(s, n, at, -1, &t, &k);  // ID
  if (rc) return rc;
  for (int32_t i = 0; i < n_allele; ++i) {
    if ((rc = bcf_typed(s, n, at, -1, &t, &k))) return rc;
    if (k > 0 && t != 7) return HBAM_ERUNTIME;  // (String) of a non-string
  }
  if ((rc = bcf_typed(s, n, at, h.n_dict, &t, &k))) return rc;  // FILTER
  for (int32_t i = 0; i < n_info; ++i) {
    if ((rc = bcf_typed(s, n, at, h.n_dict, &t, &k))) return rc;  // key
    if ((rc = bcf_typed(s, n, at, -1, &t, &k))) return rc;        // value
  }
  if ((o->n_fmt_sample >> 24) < 0 || n_allele < 1) return HBAM_ETRIBBLE;  // SitesInfoForDecoding.isValid
  return HBAM_OK;
}

// guessNextBCFPos' test at offset x of contiguous bytes (all 38 bytes it reads present)
__device__ __forceinline__ bool bcf_pred(const uint8_t* __restrict__ u, const BcfHdr& h) {
  const int64_t shared = (int64_t)ld_u32_unaligned(u), indiv = (int64_t)ld_u32_unaligned(u + 4);
  if (shared + indiv < BCF_SHORTEST) return false;
  const int32_t chrom = (int32_t)ld_u32_unaligned(u + 8), pos = (int32_t)ld_u32_unaligned(u + 12);
  if (chrom < 0 || chrom >= h.n_contig || pos < 0) return false;
  const int32_t ai = (int32_t)ld_u32_unaligned(u + 24);
  if ((ai >> 16) < 0 || (ai & 0xffff) < 0) return false;
  if ((int32_t)u[28] != h.n_sample) return false;
  const int8_t idt = (int8_t)u[32];
  if ((idt & 0x0f) != 0x07) return false;
  if ((idt & 0xf0) == 0xf0) {
    int64_t id_len;
    switch (u[33] & 0x0f) {
      case 1: id_len = u[34]; break;
      case 2: id_len = ld_u16_unaligned(u + 34); break;
      case 3: id_len = (int64_t)ld_u32_unaligned(u + 34); break;
      default: return false;
    }
    if (id_len < 15 || id_len > shared - (4 * 8 + (ai >> 16) + (int64_t)(ai & 0xffff) * 2)) return false;
  }
  return true;
}

struct BcfFmt {
  BcfHdr h;
  __device__ __forceinline__ bool plausible(const uint8_t* __restrict__ u, uint64_t x, uint64_t hard_end) const {
    if (x + 38 > hard_end) return false;
    if (!bcf_pred(u + x, h)) return false;
    return (int32_t)ld_u32_unaligned(u + x) >= BCF_MIN_SHARED && (int32_t)ld_u32_unaligned(u + x + 4) >= 0;
  }
  __device__ __forceinline__ uint64_t next(const uint8_t* __restrict__ u, uint64_t r, uint64_t hard_end) const {
    if (r + 8 > hard_end) return CHAIN_STOP;
    const int32_t ls = (int32_t)ld_u32_unaligned(u + r), li = (int32_t)ld_u32_unaligned(u + r + 4);
    if (ls < BCF_MIN_SHARED || li < 0) return CHAIN_STOP;  // cannot decode: the chain ends at it
    return r + 8 + (uint64_t)(uint32_t)ls + (uint64_t)(uint32_t)li;
  }
};

// ---- BCFRecordReader.nextKeyValue per record ----------------------------------------------
struct BcfCols {
  int32_t* status;
  int32_t* l_shared;
  int32_t* l_indiv;
  int32_t* chrom;
  int32_t* pos;
  int32_t* rlen;
  uint32_t* qual;
  int32_t* n_allele_info;
  int32_t* n_fmt_sample;
  int64_t* key;
  int64_t* rel;
};
// u: the record stream (inflated split / raw file window); records at rec_off.  The stream the
// reader sees ends at z: z_code == HBAM_OK a clean end of stream (reads past z: -1), else the
// exception of the fill that would deliver byte z.  limit: FileSplit end (uncompressed; record
// starts >= limit end the split), ~0 for BGZF.  rel = rec_off - rel_base (+ rel_add).
__global__ void k_bcf_decode(const uint8_t* __restrict__ u, uint64_t nrec, const uint64_t* __restrict__ rec_off,
                             uint64_t z, int32_t z_code, uint64_t limit, uint64_t rel_base, int64_t rel_add,
                             BcfHdr h, BcfCols c, unsigned long long* __restrict__ first_stop) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrec) return;
  const uint64_t r = rec_off[i];
  int32_t st = ST_OK;
  int32_t ls = 0, li = 0;
  BcfSite s{};
  if (r >= limit) {
    st = ST_VEND;
  } else if (r >= z) {
    st = z_code ? z_code : ST_NULL;  // peek(): -1, or the fill's exception
  } else if (r + 8 > z && z_code) {
    st = z_code;
  } else {
    uint32_t v[2] = {0, 0};
    for (int k = 0; k < 8; ++k) v[k >> 2] |= (r + k < z ? (uint32_t)u[r + k] : 0xffu) << (8 * (k & 3));
    ls = (int32_t)v[0];
    li = (int32_t)v[1];
    if (ls < 0) {
      st = HBAM_ETRIBBLE;
    } else if (ls > 0 && r + 8 + (uint64_t)ls > z) {
      st = z_code ? z_code : HBAM_ETRIBBLE;
    } else {
      BcfBytes b{u + r + 8};
      st = bcf_site(b, ls, h, &s);
      if (st == HBAM_OK) {
        if (li < 0) st = HBAM_ETRIBBLE;
        else if (li > 0 && r + 8 + (uint64_t)ls + (uint64_t)li > z) st = z_code ? z_code : HBAM_ETRIBBLE;
      }
    }
  }
  c.status[i] = st;
  if (st != ST_OK) {
    atomicMin(first_stop, (unsigned long long)i);
    return;
  }
  c.l_shared[i] = ls;
  c.l_indiv[i] = li;
  c.chrom[i] = s.chrom;
  c.pos[i] = s.pos;
  c.rlen[i] = s.rlen;
  c.qual[i] = s.qual;
  c.n_allele_info[i] = s.n_allele_info;
  c.n_fmt_sample[i] = s.n_fmt_sample;
  // BCFRecordReader.java:167-171: contigDict index (= CHROM: the dictionary is the header's
  // contig lines in order) << 32 | (long)(getStart() - 1), sign-extended
  c.key[i] = (int64_t)((uint64_t)(int64_t)s.chrom << 32 | (uint64_t)(int64_t)s.pos);
  c.rel[i] = (int64_t)(r - rel_base) + rel_add;
}

// record starts of the chain walk -> offsets in the stream (no virtual offsets for BCF)
__global__ void k_emit_rec_off(const uint64_t* __restrict__ uoff, uint32_t nblk, const uint16_t* __restrict__ rel,
                               const uint32_t* __restrict__ count, const uint64_t* __restrict__ base,
                               uint64_t* __restrict__ rec_off) {
  const uint32_t b = blockIdx.x;
  if (b >= nblk) return;
  const uint32_t n = count[b] < WALK_CAP ? count[b] : WALK_CAP;
  const uint64_t o = base[b], u0 = uoff[b];
  for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) rec_off[o + k] = u0 + rel[(uint64_t)b * WALK_CAP + k];
}

// 64 KiB segments of a raw (uncompressed BCF) stream for the chain walk
__global__ void k_raw_segments(uint64_t len, uint32_t nseg, uint64_t* __restrict__ uoff) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nseg) return;
  const uint64_t v = (uint64_t)i << 16;
  uoff[i] = v < len ? v : len;
}

// ---- BCFSplitGuesser.guessNextBCFRecordStart ---------------------------------------------------
// Byte source of the guesser: the window stream (uncompressed BCF) or the BlockCompressedInputStream
// over it (BGZF), each with its own SeekableArrayStream position.
struct BcfCur {
  GStream f;
  GBcis b;
  int bgzf;
};
__device__ __forceinline__ int32_t gs_read_skip(GStream& s, uint8_t* b, int32_t n) {
  if (s.pos == s.len) return -1;
  if ((int64_t)n > s.len - s.pos) n = (int32_t)(s.len - s.pos);
  if (b)
    for (int32_t i = 0; i < n; ++i) b[i] = s.a[s.pos + i];
  s.pos += n;
  return n;
}
// InputStream.read(byte[], 0, len) of cin; dst == nullptr skips.  *got = -1 at the end.
__device__ int32_t bc_read(BcfCur& c, uint8_t* dst, int32_t len, int32_t* got) {
  if (!c.bgzf) {
    *got = gs_read_skip(c.f, dst, len);
    return HBAM_OK;
  }
  return gb_read(c.b, c.f, dst, len, got);
}
// tribble PositionalBufferedStream without its buffer: `lead` performs the fills, `tr` reads
// the bytes the decode consumes (they were already read without error by the lead).
struct BcfPbs {
  BcfCur lead, tr;
  int32_t n_chars, next;
  int64_t position;
};
__device__ int32_t bp_fill(BcfPbs& p) {
  int32_t got;
  const int32_t rc = bc_read(p.lead, nullptr, BCF_PBS_SIZE, &got);
  if (rc) return rc;
  p.n_chars = got;
  p.next = 0;
  return HBAM_OK;
}
// peek(): *c = 0 (a byte is available) or -1
__device__ int32_t bp_peek(BcfPbs& p, int32_t* c) {
  for (;;) {
    if (p.n_chars < 0) { *c = -1; return HBAM_OK; }
    if (p.next == p.n_chars) {
      const int32_t rc = bp_fill(p);
      if (rc) return rc;
      continue;
    }
    *c = 0;
    return HBAM_OK;
  }
}
// the trailing cursor's next k bytes (k <= what the lead delivered); empty blocks read as
// short reads there too (-1, bounded by the blocks a window holds).  The lead already read these
// bytes, so an error or a cursor that stops advancing "cannot happen": it ends the decode with
// TribbleException instead of spinning.
__device__ int32_t bp_take(BcfPbs& p, uint8_t* dst, int32_t k) {
  int32_t stalls = 0;
  while (k > 0) {
    int32_t got = 0;
    const int32_t rc = bc_read(p.tr, dst, k, &got);
    if (rc) return HBAM_ETRIBBLE;
    if (got <= 0) {
      if (got == 0 || ++stalls > 16384) return HBAM_ETRIBBLE;
      continue;
    }
    if (dst) dst += got;
    k -= got;
  }
  return HBAM_OK;
}
// read(bytes, 0, len): *got = bytes or -1
__device__ int32_t bp_read(BcfPbs& p, uint8_t* dst, int32_t len, int32_t* got) {
  if (len == 0) { *got = 0; return HBAM_OK; }
  int32_t c;
  int32_t rc = bp_peek(p, &c);
  if (rc) return rc;
  if (c < 0) { *got = -1; return HBAM_OK; }
  int32_t n = 0;
  while (len - n > 0) {
    if (p.n_chars == p.next) {
      if ((rc = bp_fill(p))) return rc;
      if (p.n_chars < 0) break;
    }
    int32_t k = p.n_chars - p.next;
    if (k > len - n) k = len - n;
    if ((rc = bp_take(p, dst ? dst + n : nullptr, k))) return rc;
    p.next += k;
    n += k;
  }
  p.position += n;
  *got = n;
  return HBAM_OK;
}
// Site bytes through a copy of the trailing cursor, in order.  Only used after the lead delivered
// the whole site block, so every byte exists; a -1 is an empty BGZF block inside it (a short
// read, as for the lead), bounded by the blocks a window can hold.
struct BcfTrail {
  BcfCur c;
  int64_t pos;
  __device__ uint32_t at(int64_t i) {
    int32_t neg = 0;
    while (pos < i) {
      int32_t got;
      if (bc_read(c, nullptr, (int32_t)(i - pos), &got)) return 0xffu;
      if (got < 0) { if (++neg > 16384) return 0xffu; continue; }
      pos += got;
    }
    uint8_t v = 0xffu;
    for (;;) {
      int32_t got;
      if (bc_read(c, &v, 1, &got)) return 0xffu;
      if (got < 0) { if (++neg > 16384) return 0xffu; continue; }
      break;
    }
    ++pos;
    return v;
  }
};
// a cursor copy that owns `own` as its in-lane inflate output (the copied block moves with it)
__device__ void bc_own_scratch(BcfCur& c, uint8_t* own) {
  if (c.bgzf && c.b.cur == c.b.scratch && c.b.cur_len > 0)
    for (int32_t j = 0; j < c.b.cur_len; ++j) own[j] = c.b.scratch[j];
  if (c.b.cur == c.b.scratch) c.b.cur = own;
  c.b.scratch = own;
}

// BCF2Codec.decode over the buffered stream: 1 record, or an exception code
__device__ int32_t bcf_decode_pbs(BcfPbs& p, const BcfHdr& h, uint8_t* site_scratch) {
  uint32_t v[2] = {0, 0};
  for (int k = 0; k < 8; ++k) {  // BCF2Type.INT32.read: read() per byte, -1 & 0xFF
    int32_t c;
    int32_t rc = bp_peek(p, &c);
    if (rc) return rc;
    uint32_t byte = 0xffu;
    if (c >= 0) {
      uint8_t t = 0;
      if ((rc = bp_take(p, &t, 1))) return rc;
      byte = t;
      ++p.next;
      ++p.position;
    }
    v[k >> 2] |= byte << (8 * (k & 3));
  }
  const int32_t ls = (int32_t)v[0], li = (int32_t)v[1];
  if (ls < 0) return HBAM_ETRIBBLE;
  // the site bytes: read through the stream first (its exceptions come first), then decoded
  // from a copy of the trailing cursor taken at the block's start
  BcfTrail site{p.tr, 0};
  bc_own_scratch(site.c, site_scratch);
  for (int32_t n = 0; n < ls;) {
    int32_t got;
    const int32_t rc = bp_read(p, nullptr, ls - n, &got);
    if (rc) return rc;
    if (got < 0) return HBAM_ETRIBBLE;
    n += got;
  }
  BcfSite s;
  int32_t rc = bcf_site(site, ls, h, &s);
  if (rc) return rc;
  if (li < 0) return HBAM_ETRIBBLE;
  for (int32_t n = 0; n < li;) {
    int32_t got;
    if ((rc = bp_read(p, nullptr, li - n, &got))) return rc;
    if (got < 0) return HBAM_ETRIBBLE;
    n += got;
  }
  return 1;
}

// guessNextBCFPos :370-455: the candidate test through cin's seek/read (stale `buf` bytes on
// short reads); an IOException ends the scan (-1), other exceptions escape (*esc)
__device__ int32_t g_next_bcf(Guesser& g, BcfCur& cin, uint64_t cpv, int32_t up, int32_t csize, const BcfHdr& h,
                              int32_t* esc) {
  int32_t got, rc;
#define BSEEK(v)                                                                        \
  do {                                                                                  \
    if (!cin.bgzf) { if (!gs_seek(cin.f, (int64_t)(v))) return -1; }                   \
    else if ((rc = gb_seek(cin.b, cin.f, (v)))) { if (rc != HBAM_EIO) *esc = rc; return -1; } \
  } while (0)
#define BREAD(n)                                                                        \
  do {                                                                                  \
    if (!cin.bgzf) got = gs_read(cin.f, g.buf, (n));                                    \
    else if ((rc = gb_read(cin.b, cin.f, g.buf, (n), &got))) { if (rc != HBAM_EIO) *esc = rc; return -1; } \
  } while (0)
  for (; up + BCF_SHORTEST < csize; ++up) {
    BSEEK(cpv | (uint64_t)(int64_t)up);
    BREAD(8);
    const int64_t shared = (int64_t)(uint32_t)gbuf_i32(g, 0), indiv = (int64_t)(uint32_t)gbuf_i32(g, 4);
    if (shared + indiv < BCF_SHORTEST) continue;
    BSEEK(cpv | (uint64_t)(int64_t)(up + 8));
    BREAD(8);
    const int32_t chrom = gbuf_i32(g, 0), pos = gbuf_i32(g, 4);
    if (chrom < 0 || chrom >= h.n_contig || pos < 0) continue;
    BSEEK(cpv | (uint64_t)(int64_t)(up + 24));
    BREAD(4);
    const int32_t ai = gbuf_i32(g, 0);
    if ((ai >> 16) < 0 || (ai & 0xffff) < 0) continue;
    BSEEK(cpv | (uint64_t)(int64_t)(up + 28));
    BREAD(1);
    if ((int32_t)g.buf[0] != h.n_sample) continue;
    BSEEK(cpv | (uint64_t)(int64_t)(up + 32));
    BREAD(6);
    const int8_t idt = (int8_t)g.buf[0];
    if ((idt & 0x0f) != 0x07) continue;
    if ((idt & 0xf0) == 0xf0) {
      int64_t id_len;
      switch (g.buf[1] & 0x0f) {
        case 1: id_len = g.buf[2]; break;
        case 2: id_len = gbuf_u16(g, 2); break;
        case 3: id_len = (int64_t)(uint32_t)gbuf_i32(g, 2); break;
        default: continue;
      }
      if (id_len < 15 || id_len > shared - (4 * 8 + (ai >> 16) + (int64_t)(ai & 0xffff) * 2)) continue;
    }
    return up;
  }
#undef BSEEK
#undef BREAD
  return -1;
}

// One lane per guess; bgzf selects the compressed / uncompressed state machine.
__global__ __launch_bounds__(GUESS_WG) void k_guess_bcf(const uint64_t* __restrict__ wptr,
                                                        const int64_t* __restrict__ wlen,
                                                        const int64_t* __restrict__ beg,
                                                        const int64_t* __restrict__ end, uint32_t k, int bgzf,
                                                        BcfHdr h, uint8_t* __restrict__ scratch,
                                                        uint8_t* __restrict__ lens_scratch,
                                                        int64_t* __restrict__ out, int32_t* __restrict__ err,
                                                        const uint32_t* __restrict__ cn,
                                                        const uint64_t* __restrict__ cbase,
                                                        const uint64_t* __restrict__ cpos,
                                                        const BlockRec* __restrict__ cblk,
                                                        const uint64_t* __restrict__ cuoff,
                                                        const uint8_t* __restrict__ cubuf,
                                                        const int32_t* __restrict__ cst,
                                                        const uint32_t* __restrict__ ccrc) {
  __shared__ uint16_t s_ll[GUESS_WG * 288];
  __shared__ uint8_t s_d[GUESS_WG * 32];
  __shared__ uint32_t T[256];
  crc_table_init(T);
  const uint32_t i = blockIdx.x * GUESS_WG + threadIdx.x;
  if (i >= k) return;
  const int64_t b0 = beg[i], e0 = end[i];
  const int64_t total = g_window_total(b0, e0, wlen[i], bgzf ? BCF_BGZF_WINDOW : BCF_UNCOMP_NEEDED);
  Guesser g;
  for (int j = 0; j < 8; ++j) g.buf[j] = 0;  // ByteBuffer.allocate(8) (:96)
  g.n_ref = 0;
  g.in = GStream{(const uint8_t*)wptr[i], total, 0};
  GBcis& bz = g.bz;
  bz.block_addr = 0;
  bz.last_len = 0;
  bz.cur_len = -1;
  bz.cur_off = 0;
  bz.scratch = scratch + (uint64_t)i * 3 * 65536;
  bz.cur = bz.scratch;
  bz.wbase = b0 >= 0 ? b0 : 0;
  bz.cache.n = 0;
  if (bgzf && cn && cn[i] <= GC_CAP) {
    const uint64_t o = cbase[i];
    bz.cache.n = cn[i];
    bz.cache.pos = cpos + o;
    bz.cache.blk = cblk + o;
    bz.cache.uoff = cuoff + o;
    bz.cache.ubuf = cubuf;
    bz.cache.st = cst + o;
    bz.cache.crc = ccrc + o;
  }
  bz.s_ll = s_ll + threadIdx.x * 288;
  bz.s_d = s_d + threadIdx.x * 32;
  bz.lens = lens_scratch + (uint64_t)i * LENS_SLOT;
  bz.crc_tab = T;
  bz.check_crc = 1;  // setCheckCrcs(true) (:156)
  int32_t e = HBAM_OK;
  int64_t result = e0;
  int32_t first_end = 0;
  if (bgzf) first_end = (int32_t)(e0 - b0) < 0xffff ? (int32_t)(e0 - b0) : 0xffff;
  for (int32_t cp = 0;; ++cp) {
    int32_t cp0, block_len;
    uint64_t cp0v;
    if (bgzf) {
      int32_t ppos, psize;
      if (!g_next_bgzf(g, cp, first_end, &ppos, &psize)) break;
      cp0 = cp = ppos;
      cp0v = (uint64_t)(uint32_t)cp0 << 16;
      if (gb_seek(g.bz, g.in, cp0v)) continue;  // catch (Throwable)
      block_len = psize;
    } else {
      cp0 = 0;
      cp0v = 0;
      block_len = total > BCF_UNCOMP_NEEDED ? (int32_t)total : BCF_UNCOMP_NEEDED;
    }
    for (int32_t up = 0;; ++up) {
      BcfCur cin{g.in, g.bz, bgzf};
      int32_t esc = HBAM_OK;
      const int32_t up0 = up = g_next_bcf(g, cin, cp0v, up, block_len, h, &esc);
      g.in = cin.f;
      g.bz = cin.b;
      if (esc) { e = esc; goto done; }
      if (up0 < 0) break;
      if (bgzf) {
        if (gb_seek(g.bz, g.in, cp0v | (uint32_t)up0)) { e = HBAM_EIO; goto done; }
      } else if (!gs_seek(g.in, up0)) {
        e = HBAM_EIO;
        goto done;
      }
      // verification (:207-273): PositionalBufferedStream over cin
      BcfPbs p;
      p.lead = BcfCur{g.in, g.bz, bgzf};
      p.tr = p.lead;
      bc_own_scratch(p.tr, scratch + (uint64_t)i * 3 * 65536 + 65536);  // its own in-lane inflate output
      p.n_chars = 0;
      p.next = 0;
      p.position = 0;
      bool decoded_any = false;
      int32_t rc = HBAM_OK, c;
      int b = 0;
      if (bgzf) {
        const int32_t prev_cp = cp0;  // never updated (:216-231)
        for (;;) {
          if (b >= 2) break;
          if ((rc = bp_peek(p, &c))) break;
          if (c < 0) break;
          rc = bcf_decode_pbs(p, h, scratch + (uint64_t)i * 3 * 65536 + 2 * 65536);
          if (rc != 1) break;
          rc = HBAM_OK;
          decoded_any = true;
          const int32_t cp2 = (int32_t)(gb_tell(p.lead.b) >> 16);
          if (cp2 != prev_cp) { cp = cp2; ++b; }
        }
      } else {
        for (;;) {
          if (!(p.position - up0 < BCF_UNCOMP_NEEDED)) break;
          if ((rc = bp_peek(p, &c))) break;
          if (c < 0) break;
          rc = bcf_decode_pbs(p, h, scratch + (uint64_t)i * 3 * 65536 + 2 * 65536);
          if (rc != 1) break;
          rc = HBAM_OK;
          decoded_any = true;
        }
      }
      // cin (lead) state carries over to the next candidate
      g.in = p.lead.f;
      g.bz = p.lead.b;
      g.bz.scratch = scratch + (uint64_t)i * 3 * 65536;
      if (rc == HBAM_OK) {
        const bool short_ = bgzf ? b < 2 : (p.position - up0 < BCF_UNCOMP_NEEDED);
        if (!decoded_any && short_) continue;
      } else if (rc == HBAM_ETRUNC || rc == HBAM_ENOMEM || rc == HBAM_EEOF) {
        continue;  // FileTruncatedException / OutOfMemoryError / RuntimeEOFException
      } else if (rc == HBAM_ETRIBBLE) {
        int32_t pc = 0;
        if (decoded_any) {
          const int32_t prc = bp_peek(p, &pc);
          g.in = p.lead.f;
          g.bz = p.lead.b;
          g.bz.scratch = scratch + (uint64_t)i * 3 * 65536;
          if (prc) { e = prc; goto done; }
        }
        if (!(decoded_any && pc < 0)) continue;
      } else {
        e = rc;  // escapes guessNextBCFRecordStart
        goto done;
      }
      result = bgzf ? (int64_t)((uint64_t)(b0 + cp0) << 16 | (uint32_t)up0) : b0 + up0;
      goto done;
    }
    if (!bgzf) break;
  }
done:
  out[i] = result;
  err[i] = e;
}

}  // namespace hbam
