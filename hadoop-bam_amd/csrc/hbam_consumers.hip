// hbam_consumers.hip — read-name / CIGAR keyed consumers of the decoded records (SURVEY.md §8
// f-4), device side + C ABI.  Included at the end of hbam_capi.hip (one translation unit).
//
// Records are addressed as (ubuf, rec_off[i]): the block_size field of record i — a decoded
// split's columns (dv->ubuf, dv->rec_off) or a packed SAMRecordWritable payload buffer.
//
//  * hbam_summarize_ranges — SummarizeRecordReader (cli/plugins/chipster/Summarize.java:664-755):
//    each mapped record's CIGAR cut into reference ranges, keyed by getKey0(refIdx, centre).
//    Two kernels: per-record range count (+ the first record that raises), exclusive scan, per-
//    record emit.  Bytes: the CIGAR pool once + 21 B per range written.
//  * hbam_name_order — FixMateMapper's shuffle (FixMate.java:209-221): records ordered by
//    Text(readName) = unsigned lexicographic name bytes, proper prefix first, ties in input
//    order.  LSD over the name: a stable device radix sort (hbam_sort_keys) by length, then by
//    each 8-byte big-endian name chunk from the last to the first, composing the permutation.
//  * hbam_fixmate — FixMateReducer (FixMate.java:225-277) over the shuffle order: group heads by
//    name equality, one lane per key group replays the reducer's iterator loop (count pass,
//    scan, emit pass), then one lane per output record applies SamPairUtil.setMateInfo and
//    BAMRecordCodec.encode (restated in oracle/hbam_oracle_f4.c; parity unpinned there).
#pragma once

namespace hbam {

constexpr uint32_t F4_WG = 256;

__device__ __forceinline__ int32_t f4_ld32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint16_t f4_ld16(const uint8_t* p) { return (uint16_t)(p[0] | p[1] << 8); }
__device__ __forceinline__ void f4_st32(uint8_t* p, int32_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)((uint32_t)v >> 8);
  p[2] = (uint8_t)((uint32_t)v >> 16);
  p[3] = (uint8_t)((uint32_t)v >> 24);
}
__device__ __forceinline__ void f4_st16(uint8_t* p, uint16_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
}
__device__ __forceinline__ int32_t f4_iadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
__device__ __forceinline__ int64_t f4_key0(int32_t ref, int32_t s0) {  // BAMRecordReader.getKey0 :104-106
  return (int64_t)((uint64_t)(int64_t)ref << 32) | (int64_t)s0;
}

// Record layout bounds.  hbam_decode_split hands out a record whose variable fields do not fit
// its block_size with status OK and layout_ok = 0 (htsjdk decodes those fields lazily and throws
// only when one is read), so every consumer bounds its reads by the record's own block_size.
// f4_cigar_ok: name + CIGAR inside the record (what getCigar reads); f4_layout_ok: every field.
__device__ __forceinline__ bool f4_cigar_ok(const uint8_t* r) {
  const int64_t bs = f4_ld32(r);
  return bs >= 32 && 32 + (int64_t)r[12] + 4 * (int64_t)f4_ld16(r + 16) <= bs;
}
__device__ __forceinline__ bool f4_layout_ok(const uint8_t* r) {
  const int64_t bs = f4_ld32(r);
  const int64_t ls = f4_ld32(r + 20);
  return bs >= 32 && ls >= 0 && 32 + (int64_t)r[12] + 4 * (int64_t)f4_ld16(r + 16) + (ls + 1) / 2 + ls <= bs;
}

// ---- Summarize ------------------------------------------------------------------------------
// Walks one record's CIGAR as SummarizeRecordReader.parseCIGAR (:719-755).  EMIT=false: returns
// the range count (0xffffffff: an op code > 8, IllegalArgumentException from getCigar;
// 0xfffffffe: the CIGAR lies outside the record, the runtime exception getCigar's read of it
// raises in htsjdk; parity unpinned for that exception's class).
template <bool EMIT>
__device__ uint32_t f4_ranges(const uint8_t* r, int64_t* key, int32_t* beg, int32_t* end, uint8_t* rev,
                              uint32_t* rec, uint32_t ri) {
  const uint16_t flag = f4_ld16(r + 18);
  const int32_t ref = f4_ld32(r + 4);
  const int32_t start = f4_iadd(f4_ld32(r + 8), 1);
  if ((flag & 4u) || ref < 0 || start < 0) return 0;  // :708-709
  if (!f4_cigar_ok(r)) return 0xfffffffeu;
  const uint8_t* cig = r + 36 + r[12];
  const uint32_t nc = f4_ld16(r + 16);
  int32_t b = start, e = start;
  uint32_t k = 0;
  int64_t prev = 0;
  for (uint32_t j = 0; j < nc; ++j) {
    const uint32_t c = (uint32_t)f4_ld32(cig + 4 * j);
    const uint32_t op = c & 15u;
    const int32_t len = (int32_t)(c >> 4);
    if (op > 8u) return 0xffffffffu;
    if (op == 0u || op == 7u || op == 8u) {
      e = f4_iadd(e, len);
      continue;
    }
    if (b != e) {
      if (EMIT) {
        const int32_t ee = f4_iadd(e, -1);
        const int32_t com = (int32_t)(((int64_t)b + (int64_t)ee) / 2);
        prev = k == 0 ? f4_key0(ref, com) : (int64_t)(((uint64_t)prev >> 32) << 32) | (int64_t)com;
        key[k] = prev;
        beg[k] = b;
        end[k] = ee;
        rev[k] = (flag & 0x10u) ? 1 : 0;
        rec[k] = ri;
      }
      ++k;
      b = e;
    }
    if (op == 2u || op == 3u) {
      b = f4_iadd(b, len);
      e = b;
    }
  }
  if (b != e) {
    if (EMIT) {
      const int32_t ee = f4_iadd(e, -1);
      const int32_t com = (int32_t)(((int64_t)b + (int64_t)ee) / 2);
      prev = k == 0 ? f4_key0(ref, com) : (int64_t)(((uint64_t)prev >> 32) << 32) | (int64_t)com;
      key[k] = prev;
      beg[k] = b;
      end[k] = ee;
      rev[k] = (flag & 0x10u) ? 1 : 0;
      rec[k] = ri;
    }
    ++k;
  }
  return k;
}

// per record: range count; the first record that raises (op > 8, or a mapped record without a
// range: ranges.get(0) at :715) -> atomicMin of (record << 2 | kind) into *first_err
__global__ __launch_bounds__(F4_WG) void k_sum_count(const uint8_t* __restrict__ ubuf,
                                                     const uint64_t* __restrict__ rec_off, uint64_t n,
                                                     uint32_t* __restrict__ cnt,
                                                     unsigned long long* __restrict__ first_err) {
  const uint64_t i = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (i >= n) return;
  const uint8_t* r = ubuf + rec_off[i];
  const uint32_t k = f4_ranges<false>(r, nullptr, nullptr, nullptr, nullptr, nullptr, 0);
  uint32_t kind = 0;
  if (k == 0xffffffffu) kind = 1;
  else if (k == 0xfffffffeu) kind = 3;
  else if (k == 0 && !((f4_ld16(r + 18) & 4u) || f4_ld32(r + 4) < 0 || f4_iadd(f4_ld32(r + 8), 1) < 0)) kind = 2;
  cnt[i] = kind ? 0u : k;
  if (kind) atomicMin(first_err, (unsigned long long)(i << 2 | kind));
}

__global__ __launch_bounds__(F4_WG) void k_sum_emit(const uint8_t* __restrict__ ubuf,
                                                    const uint64_t* __restrict__ rec_off, uint64_t n,
                                                    const uint64_t* __restrict__ roff, int64_t* __restrict__ key,
                                                    int32_t* __restrict__ beg, int32_t* __restrict__ end,
                                                    uint8_t* __restrict__ rev, uint32_t* __restrict__ rec) {
  const uint64_t i = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (i >= n) return;
  const uint64_t o = roff[i];
  if (roff[i + 1] == o) return;
  f4_ranges<true>(ubuf + rec_off[i], key + o, beg + o, end + o, rev + o, rec + o, (uint32_t)i);
}

// ---- name order -------------------------------------------------------------------------
__device__ __forceinline__ uint32_t f4_name_len(const uint8_t* r) { return r[12] ? (uint32_t)r[12] - 1u : 0u; }

// name length of every record + min / max over the records
__global__ __launch_bounds__(F4_WG) void k_name_len(const uint8_t* __restrict__ ubuf,
                                                    const uint64_t* __restrict__ rec_off, uint64_t n,
                                                    int64_t* __restrict__ lenkey, uint32_t* __restrict__ mm) {
  const uint64_t i = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (i >= n) return;
  const uint32_t L = f4_name_len(ubuf + rec_off[i]);
  lenkey[i] = (int64_t)L;
  atomicMin(mm, L);
  atomicMax(mm + 1, L);
}

// key of position i = 8-byte big-endian chunk c of the name of record perm[i] (zero padded),
// sign bit flipped so that hbam_sort_keys' signed order is the chunk's unsigned order
__global__ __launch_bounds__(F4_WG) void k_name_chunk(const uint8_t* __restrict__ ubuf,
                                                      const uint64_t* __restrict__ rec_off,
                                                      const uint32_t* __restrict__ perm, uint64_t n,
                                                      uint32_t c, int64_t* __restrict__ key) {
  const uint64_t i = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (i >= n) return;
  const uint8_t* r = ubuf + rec_off[perm ? perm[i] : (uint32_t)i];
  const uint32_t L = f4_name_len(r);
  const uint8_t* nm = r + 36;
  uint64_t v = 0;
#pragma unroll
  for (uint32_t b = 0; b < 8; ++b) {
    const uint32_t j = 8u * c + b;
    v = v << 8 | (j < L ? nm[j] : 0u);
  }
  key[i] = (int64_t)(v ^ 0x8000000000000000ull);
}

// first record whose fields do not fit its block_size (FixMateMapper reads every record's name,
// the reducer re-encodes every field) -> atomicMin into *first_err
__global__ __launch_bounds__(F4_WG) void k_layout_check(const uint8_t* __restrict__ ubuf,
                                                        const uint64_t* __restrict__ rec_off, uint64_t n,
                                                        unsigned long long* __restrict__ first_err) {
  const uint64_t i = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (i < n && !f4_layout_ok(ubuf + rec_off[i])) atomicMin(first_err, (unsigned long long)i);
}

__global__ __launch_bounds__(F4_WG) void k_iota(uint64_t n, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (i < n) out[i] = (uint32_t)i;
}

// perm_out[i] = perm_in[p[i]]
__global__ __launch_bounds__(F4_WG) void k_perm_compose(const uint32_t* __restrict__ perm_in,
                                                        const uint32_t* __restrict__ p, uint64_t n,
                                                        uint32_t* __restrict__ perm_out) {
  const uint64_t i = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (i < n) perm_out[i] = perm_in ? perm_in[p[i]] : p[i];
}

// ---- FixMate ------------------------------------------------------------------------------
__device__ bool f4_name_eq(const uint8_t* a, const uint8_t* b) {
  const uint32_t la = f4_name_len(a), lb = f4_name_len(b);
  if (la != lb) return false;
  for (uint32_t k = 0; k < la; ++k)
    if (a[36 + k] != b[36 + k]) return false;
  return true;
}

__global__ __launch_bounds__(F4_WG) void k_fm_heads(const uint8_t* __restrict__ ubuf,
                                                    const uint64_t* __restrict__ rec_off,
                                                    const uint32_t* __restrict__ perm, uint64_t n,
                                                    uint32_t* __restrict__ head) {
  const uint64_t i = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (i >= n) return;
  head[i] = (i == 0 || !f4_name_eq(ubuf + rec_off[perm[i]], ubuf + rec_off[perm[i - 1]])) ? 1u : 0u;
}

__global__ __launch_bounds__(F4_WG) void k_fm_gstart(const uint32_t* __restrict__ head,
                                                     const uint64_t* __restrict__ hpos, uint64_t n,
                                                     uint64_t* __restrict__ gstart) {
  const uint64_t i = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (i < n && head[i]) gstart[hpos[i]] = i;
  if (i == 0) gstart[hpos[n]] = n;
}

// FixMateReducer.reduce (:230-277) for one key group [g0, g1) of the shuffle order.  Output
// entry: src record, mate record (or ~0u: written as read), role (1 = rec1 of setMateInfo,
// 2 = rec2).  EMIT=false: count only.
template <bool EMIT>
__device__ uint32_t f4_reduce(const uint8_t* __restrict__ ubuf, const uint64_t* __restrict__ rec_off,
                              const uint32_t* __restrict__ perm, uint64_t g0, uint64_t g1,
                              uint32_t* src, uint32_t* mate, uint8_t* role) {
  uint32_t k = 0;
  uint64_t it = g0;
  auto put = [&](uint32_t s, uint32_t m, uint8_t ro) {
    if (EMIT) {
      src[k] = s;
      mate[k] = m;
      role[k] = ro;
    }
    ++k;
  };
  auto secondary = [&](uint32_t ri) { return (f4_ld16(ubuf + rec_off[ri] + 18) & 0x100u) != 0; };
  while (it < g1) {
    const uint32_t a = perm[it++];
    if (secondary(a)) {
      put(a, ~0u, 0);
      continue;
    }
    bool have_b = false;
    uint32_t b = 0;
    while (it < g1) {
      b = perm[it++];
      have_b = true;
      if (!secondary(b)) break;
      put(b, ~0u, 0);
    }
    if (!have_b) {
      put(a, ~0u, 0);
      break;
    }
    put(a, b, 1);
    put(b, a, 2);
  }
  return k;
}

__global__ __launch_bounds__(F4_WG) void k_fm_plan(const uint8_t* __restrict__ ubuf,
                                                   const uint64_t* __restrict__ rec_off,
                                                   const uint32_t* __restrict__ perm,
                                                   const uint64_t* __restrict__ gstart, uint64_t ng,
                                                   uint32_t* __restrict__ gcnt, const uint64_t* __restrict__ gout,
                                                   uint32_t* __restrict__ src, uint32_t* __restrict__ mate,
                                                   uint8_t* __restrict__ role) {
  const uint64_t g = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (g >= ng) return;
  if (!gout) {
    gcnt[g] = f4_reduce<false>(ubuf, rec_off, perm, gstart[g], gstart[g + 1], nullptr, nullptr, nullptr);
  } else {
    const uint64_t o = gout[g];
    f4_reduce<true>(ubuf, rec_off, perm, gstart[g], gstart[g + 1], src + o, mate + o, role + o);
  }
}

// SAMRecord state of one record during setMateInfo (mirrors fm_rec of the oracle)
struct F4Rec {
  const uint8_t* r;
  int32_t ref, pos, nref, npos, tlen;
  uint32_t flag;
  int32_t mq;  // -1 keep, -2 remove, >= 0 set
  bool bin_stale;
};
__device__ void f4_load(F4Rec& f, const uint8_t* r) {
  f.r = r;
  f.ref = f4_ld32(r + 4);
  f.pos = f4_ld32(r + 8);
  f.flag = f4_ld16(r + 18);
  f.nref = f4_ld32(r + 24);
  f.npos = f4_ld32(r + 28);
  f.tlen = f4_ld32(r + 32);
  f.mq = -1;
  f.bin_stale = false;
}
__device__ __forceinline__ bool f4_unm(const F4Rec& f) { return (f.flag & 4u) != 0; }
__device__ __forceinline__ bool f4_neg(const F4Rec& f) { return (f.flag & 0x10u) != 0; }
__device__ __forceinline__ int32_t f4_start(const F4Rec& f) { return f4_iadd(f.pos, 1); }
__device__ __forceinline__ void f4_mflags(F4Rec& f, bool neg, bool unm) {
  f.flag = (f.flag & ~0x28u) | (neg ? 0x20u : 0u) | (unm ? 8u : 0u);
}
__device__ int32_t f4_end(const F4Rec& f) {  // getAlignmentEnd
  if (f4_unm(f)) return 0;
  const uint8_t* cig = f.r + 36 + f.r[12];
  int32_t s = 0;
  const uint32_t nc = f4_ld16(f.r + 16);
  for (uint32_t j = 0; j < nc; ++j) {
    const uint32_t c = (uint32_t)f4_ld32(cig + 4 * j), op = c & 15u;
    if (op == 0u || op == 2u || op == 3u || op == 7u || op == 8u) s = f4_iadd(s, (int32_t)(c >> 4));
  }
  return f4_iadd(f4_iadd(f4_start(f), s), -1);
}
__device__ void f4_set_mate_info(F4Rec& a, F4Rec& b) {  // SamPairUtil.setMateInfo(a, b, header)
  if (!f4_unm(a) && !f4_unm(b)) {
    a.nref = b.ref;
    a.npos = b.pos;
    f4_mflags(a, f4_neg(b), false);
    a.mq = b.r[13];
    b.nref = a.ref;
    b.npos = a.pos;
    f4_mflags(b, f4_neg(a), false);
    b.mq = a.r[13];
  } else if (f4_unm(a) && f4_unm(b)) {
    const bool na = f4_neg(a), nb = f4_neg(b);
    a.ref = b.ref = -1;
    a.pos = b.pos = -1;
    a.bin_stale = b.bin_stale = true;
    a.nref = b.nref = -1;
    a.npos = b.npos = -1;
    f4_mflags(a, nb, true);
    f4_mflags(b, na, true);
    a.mq = b.mq = -2;
    a.tlen = b.tlen = 0;
  } else {
    F4Rec& m = f4_unm(a) ? b : a;
    F4Rec& u = f4_unm(a) ? a : b;
    u.ref = m.ref;
    u.pos = m.pos;
    u.bin_stale = true;
    m.nref = u.ref;
    m.npos = u.pos;
    f4_mflags(m, f4_neg(u), true);
    m.mq = -2;
    m.tlen = 0;
    u.nref = m.ref;
    u.npos = m.pos;
    f4_mflags(u, f4_neg(m), false);
    u.mq = m.r[13];
    u.tlen = 0;
  }
  int32_t is = 0;  // computeInsertSize(a, b)
  if (!f4_unm(a) && !f4_unm(b) && a.ref == b.ref) {
    const int32_t p1 = f4_neg(a) ? f4_end(a) : f4_start(a);
    const int32_t p2 = f4_neg(b) ? f4_end(b) : f4_start(b);
    is = f4_iadd(f4_iadd(p2, -p1), p2 >= p1 ? 1 : -1);
  }
  a.tlen = is;
  b.tlen = f4_iadd(0, -is);
}
__device__ __forceinline__ char f4_int_type(int64_t v) {  // BinaryTagCodec.getIntegerType
  if (v > 2147483647LL) return 'I';
  if (v > 65535) return 'i';
  if (v > 255) return 'S';
  if (v > 127) return 'C';
  if (v >= -128) return 'c';
  if (v >= -32768) return 's';
  return 'i';
}
__device__ __forceinline__ uint32_t f4_tsz(char t) { return t == 'c' || t == 'C' ? 1u : t == 's' || t == 'S' ? 2u : 4u; }
__device__ __forceinline__ void f4_put_tag(uint8_t* d, uint8_t t0, uint8_t t1, char ty, int64_t v) {
  d[0] = t0;
  d[1] = t1;
  d[2] = (uint8_t)ty;
  const uint32_t s = f4_tsz(ty);
  for (uint32_t k = 0; k < s; ++k) d[3 + k] = (uint8_t)((uint64_t)v >> (8 * k));
}
__device__ int64_t f4_aux_vsize(const uint8_t* p, uint64_t avail, char t) {
  switch (t) {
    case 'A': case 'c': case 'C': return 1;
    case 's': case 'S': return 2;
    case 'i': case 'I': case 'f': return 4;
    case 'Z': case 'H':
      for (uint64_t k = 0; k < avail; ++k)
        if (p[k] == 0) return (int64_t)k + 1;
      return -1;
    case 'B': {
      if (avail < 5) return -1;
      const char st = (char)p[0];
      const uint32_t cnt = (uint32_t)f4_ld32(p + 1);
      const uint32_t es = (st == 'c' || st == 'C') ? 1u : (st == 's' || st == 'S') ? 2u
                          : (st == 'i' || st == 'I' || st == 'f') ? 4u : 0u;
      if (!es) return -1;
      return 5 + (int64_t)cnt * es;
    }
    default: return -1;
  }
}
__device__ int64_t f4_aux_int(const uint8_t* p, char t) {
  switch (t) {
    case 'c': return (int8_t)p[0];
    case 'C': return p[0];
    case 's': return (int16_t)f4_ld16(p);
    case 'S': return f4_ld16(p);
    case 'i': return f4_ld32(p);
    default: return (uint32_t)f4_ld32(p);
  }
}
__device__ int f4_reg2bin(int beg, int end) {
  --end;
  if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
  if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
  if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
  if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
  if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
  return 0;
}
// BAMRecordCodec.encode of a record: untouched (mate == ~0u) -> its own bytes; paired -> re-
// serialized after setMateInfo (see oracle fm_encode).  dst == nullptr: length only.  Returns
// the payload length or -1 (attributes do not parse: SAMFormatException).
__device__ int64_t f4_encode(const uint8_t* __restrict__ ubuf, const uint64_t* __restrict__ rec_off,
                             uint32_t s, uint32_t m, uint8_t ro, uint8_t* __restrict__ dst) {
  const uint8_t* r = ubuf + rec_off[s];
  const int32_t bs = f4_ld32(r);
  if (m == ~0u) {
    if (dst)
      for (int64_t k = 0; k < (int64_t)bs + 4; ++k) dst[k] = r[k];
    return (int64_t)bs + 4;
  }
  F4Rec a, b;
  f4_load(a, ubuf + rec_off[ro == 1 ? s : m]);
  f4_load(b, ubuf + rec_off[ro == 1 ? m : s]);
  f4_set_mate_info(a, b);
  const F4Rec& f = ro == 1 ? a : b;
  const uint32_t lrn = r[12], nc = f4_ld16(r + 16);
  const int32_t lseq = f4_ld32(r + 20);
  const uint64_t ls = lseq > 0 ? (uint64_t)lseq : 0;
  const uint64_t head = 36 + lrn + 4ull * nc, sq = (ls + 1) / 2;
  const uint8_t* aux = r + head + sq + ls;
  const uint64_t aux_len = (uint64_t)bs + 4 - (head + sq + ls);
  uint64_t o = head + sq + ls;
  bool mq_done = false;
  uint64_t p = 0;
  while (p < aux_len) {
    if (aux_len - p < 3) return -1;
    const uint8_t t0 = aux[p], t1 = aux[p + 1];
    const char ty = (char)aux[p + 2];
    const int64_t vs = f4_aux_vsize(aux + p + 3, aux_len - p - 3, ty);
    if (vs < 0 || (uint64_t)vs > aux_len - p - 3) return -1;
    const bool is_mc = t0 == 'M' && t1 == 'C', is_mq = t0 == 'M' && t1 == 'Q';
    if (is_mc) {
      // removed (setMateCigar == false)
    } else if (is_mq && f.mq != -1) {
      if (f.mq >= 0) {
        const char nt = f4_int_type(f.mq);
        if (dst) f4_put_tag(dst + o, 'M', 'Q', nt, f.mq);
        o += 3 + f4_tsz(nt);
      }
      mq_done = true;
    } else if (ty == 'c' || ty == 'C' || ty == 's' || ty == 'S' || ty == 'i' || ty == 'I') {
      const int64_t v = f4_aux_int(aux + p + 3, ty);
      const char nt = f4_int_type(v);
      if (dst) f4_put_tag(dst + o, t0, t1, nt, v);
      o += 3 + f4_tsz(nt);
    } else {
      if (dst)
        for (uint64_t k = 0; k < 3 + (uint64_t)vs; ++k) dst[o + k] = aux[p + k];
      o += 3 + (uint64_t)vs;
    }
    p += 3 + (uint64_t)vs;
  }
  if (!mq_done && f.mq >= 0) {
    const char nt = f4_int_type(f.mq);
    if (dst) f4_put_tag(dst + o, 'M', 'Q', nt, f.mq);
    o += 3 + f4_tsz(nt);
  }
  if (dst) {
    for (uint64_t k = 0; k < head; ++k) dst[k] = r[k];
    f4_st32(dst, (int32_t)(o - 4));
    f4_st32(dst + 4, f.ref);
    f4_st32(dst + 8, f.pos);
    uint16_t bin = f4_ld16(r + 14);
    if (f.ref < 0) {
      bin = 0;
    } else if (f.bin_stale) {  // SAMRecord.computeIndexingBin
      const int32_t s0 = f.pos;
      int32_t e = f4_end(f);
      if (e <= 0) e = f4_iadd(s0, 1);
      bin = (uint16_t)f4_reg2bin(s0, e);
    }
    f4_st16(dst + 14, bin);
    f4_st16(dst + 18, (uint16_t)f.flag);
    f4_st32(dst + 24, f.nref);
    f4_st32(dst + 28, f.npos);
    f4_st32(dst + 32, f.tlen);
    for (uint64_t k = 0; k < sq; ++k) dst[head + k] = r[head + k];
    if (ls & 1u) dst[head + sq - 1] &= 0xf0u;
    const bool noqual = ls && r[head + sq] == 0xffu;
    for (uint64_t k = 0; k < ls; ++k) dst[head + sq + k] = noqual ? 0xffu : r[head + sq + k];
  }
  return (int64_t)o;
}

// per output record: payload length (pass 1) or the payload (pass 2); the first output whose
// attributes do not parse -> atomicMin into *first_err
__global__ __launch_bounds__(F4_WG) void k_fm_encode(const uint8_t* __restrict__ ubuf,
                                                     const uint64_t* __restrict__ rec_off, uint64_t nout,
                                                     const uint32_t* __restrict__ src, const uint32_t* __restrict__ mate,
                                                     const uint8_t* __restrict__ role, uint32_t* __restrict__ lens,
                                                     const uint64_t* __restrict__ ooff, uint8_t* __restrict__ out,
                                                     unsigned long long* __restrict__ first_err) {
  const uint64_t i = (uint64_t)blockIdx.x * F4_WG + threadIdx.x;
  if (i >= nout) return;
  if (!out) {
    const int64_t L = f4_encode(ubuf, rec_off, src[i], mate[i], role[i], nullptr);
    lens[i] = L < 0 ? 0u : (uint32_t)L;
    if (L < 0) atomicMin(first_err, (unsigned long long)i);
  } else {
    if (ooff[i + 1] == ooff[i]) return;
    f4_encode(ubuf, rec_off, src[i], mate[i], role[i], out + ooff[i]);
  }
}

}  // namespace hbam

// ---- C ABI ------------------------------------------------------------------------------------
namespace {
int f4_check_records(hbam_ctx* c, const uint8_t* ubuf, const uint64_t* rec_off, uint64_t n) {
  if (n && (!ubuf || !rec_off)) return set_err(c, HBAM_EINVAL, "records: null ubuf / rec_off");
  if (n > 0xffffffffull) return set_err(c, HBAM_EINVAL, "records: n > 2^32-1");
  return HBAM_OK;
}
}  // namespace

extern "C" int hbam_summarize_ranges(hbam_ctx* c, const hbam_columns* dv, hbam_ranges* out) {
  if (!c || !dv || !out) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  const uint64_t n = dv->n_records;
  int rc;
  if ((rc = f4_check_records(c, dv->ubuf, dv->rec_off, n))) return rc;
  *out = hbam_ranges{};
  out->status = dv->status == HBAM_EMORE ? HBAM_OK : dv->status;
  if (n == 0) return HBAM_OK;
  uint32_t* cnt;
  uint64_t *roff, *err;
  if ((rc = ensure(c, B_F4_CNT, n + 1, &cnt)) || (rc = ensure(c, B_F4_OFF, n + 1, &roff)) ||
      (rc = ensure(c, B_F4_ERR, 2, &err)))
    return rc;
  HIPCHK(c, hipEventRecord(c->ev[9], c->stream));
  HIPCHK(c, hipMemsetAsync(err, 0xff, 8, c->stream));
  k_sum_count<<<grid_for(n, F4_WG), F4_WG, 0, c->stream>>>(dv->ubuf, dv->rec_off, n, cnt,
                                                          (unsigned long long*)err);
  HIPCHK(c, hipGetLastError());
  uint64_t total = 0;
  if ((rc = scan_exclusive(c, cnt, n, roff, &total))) return rc;
  uint64_t e = 0;
  HIPCHK(c, copy_sync(c, &e, err, 8, hipMemcpyDeviceToHost));
  uint64_t nrec = n;
  if (e != ~0ull) {  // a record raises: the ranges of the records before it, then its exception
    nrec = e >> 2;
    out->status = (e & 3u) == 1u ? HBAM_EREFID : (e & 3u) == 3u ? HBAM_EFORMAT : HBAM_EINDEX;
    HIPCHK(c, copy_sync(c, &total, roff + nrec, 8, hipMemcpyDeviceToHost));
  }
  int64_t* key;
  int32_t *beg, *end;
  uint8_t* rev;
  uint32_t* rec;
  if ((rc = ensure(c, B_F4_KEY, total + 1, &key)) || (rc = ensure(c, B_F4_BEG, total + 1, &beg)) ||
      (rc = ensure(c, B_F4_END, total + 1, &end)) || (rc = ensure(c, B_F4_REV, total + 1, &rev)) ||
      (rc = ensure(c, B_F4_REC, total + 1, &rec)))
    return rc;
  if (nrec)
    k_sum_emit<<<grid_for(nrec, F4_WG), F4_WG, 0, c->stream>>>(dv->ubuf, dv->rec_off, nrec, roff, key, beg,
                                                               end, rev, rec);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->ev[10], c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->timing = hbam_timing{};
  c->timing.total_ms = ev_ms(c, 9, 10);
  c->timing.n_records = n;
  out->n = total;
  out->key = key;
  out->beg = beg;
  out->end = end;
  out->rev = rev;
  out->record = rec;
  return HBAM_OK;
}

extern "C" int hbam_name_order(hbam_ctx* c, const uint8_t* ubuf, const uint64_t* rec_off, uint64_t n,
                               uint32_t* perm) {
  if (!c || (n && !perm)) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = f4_check_records(c, ubuf, rec_off, n))) return rc;
  if (n == 0) return HBAM_OK;
  int64_t* key;
  uint32_t *p, *tmp, *mm;
  if ((rc = ensure(c, B_F4_NKEY, n, &key)) || (rc = ensure(c, B_F4_NP, n, &p)) ||
      (rc = ensure(c, B_F4_NTMP, n, &tmp)) || (rc = ensure(c, B_F4_MM, 2, &mm)))
    return rc;
  const uint32_t init[2] = {0xffffffffu, 0u};
  HIPCHK(c, hipMemcpyAsync(mm, init, 8, hipMemcpyHostToDevice, c->stream));
  k_name_len<<<grid_for(n, F4_WG), F4_WG, 0, c->stream>>>(ubuf, rec_off, n, key, mm);
  HIPCHK(c, hipGetLastError());
  uint32_t h[2];
  HIPCHK(c, copy_sync(c, h, mm, 8, hipMemcpyDeviceToHost));
  // LSD: length (the proper-prefix rule), then the 8-byte chunks from the last to the first
  bool have = false;
  if (h[0] != h[1]) {
    if ((rc = hbam_sort_keys(c, key, n, nullptr, perm))) return rc;
    have = true;
  }
  const uint32_t nch = (h[1] + 7u) / 8u;
  for (int ch = (int)nch - 1; ch >= 0; --ch) {
    // (no order yet: position i is record i)
    k_name_chunk<<<grid_for(n, F4_WG), F4_WG, 0, c->stream>>>(ubuf, rec_off, have ? perm : nullptr, n,
                                                             (uint32_t)ch, key);
    HIPCHK(c, hipGetLastError());
    if ((rc = hbam_sort_keys(c, key, n, nullptr, p))) return rc;
    k_perm_compose<<<grid_for(n, F4_WG), F4_WG, 0, c->stream>>>(have ? perm : nullptr, p, n, tmp);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(perm, tmp, n * 4, hipMemcpyDeviceToDevice, c->stream));
    have = true;
  }
  if (!have) {  // every name empty: input order
    k_iota<<<grid_for(n, F4_WG), F4_WG, 0, c->stream>>>(n, perm);
    HIPCHK(c, hipGetLastError());
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return HBAM_OK;
}

extern "C" int hbam_fixmate(hbam_ctx* c, const uint8_t* ubuf, const uint64_t* rec_off, uint64_t n,
                            hbam_fixmate_run* out) {
  if (!c || !out) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = f4_check_records(c, ubuf, rec_off, n))) return rc;
  *out = hbam_fixmate_run{};
  if (n == 0) return HBAM_OK;
  uint32_t *perm, *head;
  uint64_t *hpos, *gstart, *err;
  if ((rc = ensure(c, B_F4_PERM, n, &perm)) || (rc = ensure(c, B_F4_CNT, n + 1, &head)) ||
      (rc = ensure(c, B_F4_OFF, n + 1, &hpos)) || (rc = ensure(c, B_F4_GST, n + 1, &gstart)) ||
      (rc = ensure(c, B_F4_ERR, 2, &err)))
    return rc;
  HIPCHK(c, hipEventRecord(c->ev[13], c->stream));
  {
    // a record whose fields overrun its block_size fails the job in the mapper (getReadName /
    // the lazy field decode throws), before any output: no outputs, SAMFormatException
    HIPCHK(c, hipMemsetAsync(err, 0xff, 8, c->stream));
    k_layout_check<<<grid_for(n, F4_WG), F4_WG, 0, c->stream>>>(ubuf, rec_off, n, (unsigned long long*)err);
    HIPCHK(c, hipGetLastError());
    uint64_t e = 0;
    HIPCHK(c, copy_sync(c, &e, err, 8, hipMemcpyDeviceToHost));
    if (e != ~0ull) {
      out->status = HBAM_EFORMAT;
      return HBAM_OK;
    }
  }
  if ((rc = hbam_name_order(c, ubuf, rec_off, n, perm))) return rc;
  k_fm_heads<<<grid_for(n, F4_WG), F4_WG, 0, c->stream>>>(ubuf, rec_off, perm, n, head);
  HIPCHK(c, hipGetLastError());
  uint64_t ng = 0;
  if ((rc = scan_exclusive(c, head, n, hpos, &ng))) return rc;
  k_fm_gstart<<<grid_for(n, F4_WG), F4_WG, 0, c->stream>>>(head, hpos, n, gstart);
  HIPCHK(c, hipGetLastError());
  uint32_t* gcnt;
  uint64_t* gout;
  if ((rc = ensure(c, B_F4_GCNT, ng + 1, &gcnt)) || (rc = ensure(c, B_F4_GOUT, ng + 1, &gout))) return rc;
  k_fm_plan<<<grid_for(ng, F4_WG), F4_WG, 0, c->stream>>>(ubuf, rec_off, perm, gstart, ng, gcnt, nullptr,
                                                          nullptr, nullptr, nullptr);
  HIPCHK(c, hipGetLastError());
  uint64_t nout = 0;
  if ((rc = scan_exclusive(c, gcnt, ng, gout, &nout))) return rc;
  uint32_t *src, *mate, *lens;
  uint8_t* role;
  uint64_t* ooff;
  if ((rc = ensure(c, B_F4_SRC, nout + 1, &src)) || (rc = ensure(c, B_F4_MATE, nout + 1, &mate)) ||
      (rc = ensure(c, B_F4_ROLE, nout + 1, &role)) || (rc = ensure(c, B_F4_LENS, nout + 1, &lens)) ||
      (rc = ensure(c, B_F4_OOFF, nout + 1, &ooff)))
    return rc;
  k_fm_plan<<<grid_for(ng, F4_WG), F4_WG, 0, c->stream>>>(ubuf, rec_off, perm, gstart, ng, gcnt, gout, src,
                                                          mate, role);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemsetAsync(err, 0xff, 8, c->stream));
  k_fm_encode<<<grid_for(nout, F4_WG), F4_WG, 0, c->stream>>>(ubuf, rec_off, nout, src, mate, role, lens,
                                                             nullptr, nullptr, (unsigned long long*)err);
  HIPCHK(c, hipGetLastError());
  uint64_t e = 0;
  HIPCHK(c, copy_sync(c, &e, err, 8, hipMemcpyDeviceToHost));
  out->status = HBAM_OK;
  if (e != ~0ull) {  // the job fails at this write: the outputs before it stand
    nout = e;
    out->status = HBAM_EFORMAT;
  }
  uint64_t bytes = 0;
  if ((rc = scan_exclusive(c, lens, nout, ooff, &bytes))) return rc;
  uint8_t* pay;
  if ((rc = ensure(c, B_F4_PAY, bytes + 1, &pay))) return rc;
  if (nout)
    k_fm_encode<<<grid_for(nout, F4_WG), F4_WG, 0, c->stream>>>(ubuf, rec_off, nout, src, mate, role, lens,
                                                               ooff, pay, (unsigned long long*)err);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->ev[14], c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->timing = hbam_timing{};
  c->timing.total_ms = ev_ms(c, 13, 14);
  c->timing.n_records = n;
  out->n = nout;
  out->payload_bytes = bytes;
  out->src = src;
  out->mate = mate;
  out->offsets = ooff;
  out->payload = pay;
  out->n_groups = ng;
  return HBAM_OK;
}
