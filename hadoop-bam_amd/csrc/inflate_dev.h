// inflate_dev.h — raw DEFLATE (RFC 1951) decoder for one BGZF block per lane, gfx950.
//
// Replaces [htsjdk] BlockGunzipper.unzipBlock -> java.util.zip.Inflater (JDK zlib) for
// the BAM read path (BAMRecordReader.java:133-143 -> BlockCompressedInputStream.readBlock).
// The observable contract is zlib 1.2.11's, as java.util.zip.Inflater.inflate() drives it:
// ONE inflate(Z_PARTIAL_FLUSH) call with avail_out = ISIZE.  So:
//   * output stops at ISIZE bytes; zlib still decodes the symbol(s) that follow until one
//     would need an output byte, and reports format errors found on the way;
//   * running out of input is not an error (short output -> SAMFormatException upstream);
//   * errors (-> DataFormatException) are exactly zlib's: invalid block type, stored
//     LEN/NLEN mismatch, HLIT>286/HDIST>30, over-subscribed or incomplete code sets
//     (incomplete allowed only for a single 1-bit lit/len or distance code), code-length
//     repeat errors, missing end-of-block code, invalid lit/len (286,287) or distance
//     (30,31) symbols, distance too far back.  An all-zero code-length code decodes every
//     code length as 0 using 1 bit (zlib's CODELENS does not check the invalid marker).
//
// Design (SIMT, MI355X): each lane owns one BGZF block.  Canonical Huffman decode keeps,
// per alphabet, the 15 left-justified code-range limits and index offsets in VGPRs
// (statically unrolled compare chain: code length = 1 + #limits <= v), and only the
// symbol permutation in LDS (u16 x 288 + u8 x 32 per lane = 608 B).  Code lengths of a
// dynamic header live in a per-block global scratch slot (320 B).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hbam {

enum : int32_t {
  INF_OK = 0,
  INF_SHORT = 1,  // fewer than ISIZE bytes produced ("Did not inflate expected amount")
  INF_DATA = 2,   // zlib Z_DATA_ERROR (DataFormatException)
};

// The batched inflate's input loads and token stores use the default cache policy.  Measured and
// dropped (round 2): non-temporal token stores cut the Huffman pass's input FETCH to C (6.1 ->
// 2.1 GB per 2 GB decode), but their write acknowledgements are slow and every epoch's
// `s_waitcnt vmcnt(0)` (vmcnt counts stores too on CDNA) waits for the last iteration's stores:
// 105 -> 70 ms at 10 GB with plain stores (profiles/r02/s2/ab_store_epoch_10g.txt); non-temporal
// input loads 69.9 vs 70 ms.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_quad(const uint4* p) {
  return *p;
}
__device__ __forceinline__ void st_out(uint4* p, uint4 v) {
  *p = v;
}
__device__ __forceinline__ void st_out(uint32_t* p, uint32_t v) {
  *p = v;
}

struct BitIn {
  const uint4* qp;     // next 16-byte quad to load
  uint4 q, qn;         // current and prefetched quad
  uint32_t qi;         // next dword of q to consume (0..4)
  uint64_t bb;         // bit buffer (LSB first)
  uint32_t bc;         // valid bits in bb
  uint32_t consumed;   // bits consumed from the stream
  uint32_t total;      // 8 * deflated bytes
};

__device__ __forceinline__ uint32_t quad_word(const uint4& q, uint32_t i) {
  return i == 0 ? q.x : i == 1 ? q.y : i == 2 ? q.z : q.w;
}
// Input arrives 16 bytes per load, one quad prefetched ahead, so a refill rarely waits.
__device__ __forceinline__ void br_init(BitIn& b, const uint8_t* p, uint32_t nbytes) {
  const uintptr_t a = (uintptr_t)p & 15u;
  b.qp = (const uint4*)(p - a);
  b.q = ld_quad(b.qp);
  b.qn = ld_quad(b.qp + 1);
  b.qp += 2;
  const uint32_t w = quad_word(b.q, (uint32_t)(a >> 2));
  const uint32_t sh = 8u * (uint32_t)(a & 3u);
  b.bb = (uint64_t)(w >> sh);
  b.bc = 32u - sh;
  b.qi = (uint32_t)(a >> 2) + 1u;
  b.consumed = 0;
  b.total = nbytes * 8u;
}
__device__ __forceinline__ void br_refill(BitIn& b) {
  if (b.bc <= 32u) {
    if (b.qi == 4u) {
      b.q = b.qn;
      b.qn = ld_quad(b.qp);
      ++b.qp;
      b.qi = 0;
    }
    b.bb |= (uint64_t)quad_word(b.q, b.qi) << b.bc;
    ++b.qi;
    b.bc += 32u;
  }
}
__device__ __forceinline__ uint32_t br_avail(const BitIn& b) { return b.total - b.consumed; }
__device__ __forceinline__ uint32_t br_peek(const BitIn& b, uint32_t n) {
  return (uint32_t)b.bb & ((1u << n) - 1u);  // n <= 16 here
}
__device__ __forceinline__ void br_drop(BitIn& b, uint32_t n) {
  b.bb >>= n;
  b.bc -= n;
  b.consumed += n;
}
// next 15 stream bits as a left-justified MSB-first code value
__device__ __forceinline__ uint32_t br_rev15(const BitIn& b) {
  return __builtin_bitreverse32((uint32_t)b.bb) >> 17;
}

struct Huff {
  uint32_t lim[15];  // lim[l-1] = (first_l + count_l) << (15-l)
  int32_t doff[15];  // off[l-1] = (#codes shorter than l) - first_l, stored as deltas:
                     // doff[0] = off[0], doff[k] = off[k] - off[k-1] (an add chain keeps the
                     // compiler from rewriting the select chain into a scratch-indexed load)
  uint32_t empty;    // no codes at all (zlib max == 0)
  uint32_t hlim[15]; // lit/len only: left-justified start of the length-l codes whose symbols
                     // are >= 256 (canonical order puts them last within a length), so a u8
                     // symbol table plus one compare recovers the 9-bit symbol
};

// code length / symbol index for a left-justified 15-bit value; returns false if invalid
__device__ __forceinline__ bool huff_lookup(const Huff& h, uint32_t v, uint32_t& L, int32_t& idx) {
  uint32_t l = 1;
  int32_t o = h.doff[0];
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const bool ge = v >= h.lim[k];
    l += ge ? 1u : 0u;
    o += ge ? h.doff[k + 1] : 0;
  }
  L = l;
  idx = o + (int32_t)(v >> (15u - l));
  return v < h.lim[14];
}
// huff_lookup plus the symbol's bit 8 (lit/len tables built with kind 1)
__device__ __forceinline__ bool huff_lookup_hi(const Huff& h, uint32_t v, uint32_t& L, int32_t& idx,
                                               uint32_t& hi) {
  uint32_t l = 1;
  int32_t o = h.doff[0];
  uint32_t t = h.hlim[0];
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const bool ge = v >= h.lim[k];
    l += ge ? 1u : 0u;
    o += ge ? h.doff[k + 1] : 0;
    t = ge ? h.hlim[k + 1] : t;
  }
  L = l;
  idx = o + (int32_t)(v >> (15u - l));
  hi = v >= t ? 256u : 0u;
  return v < h.lim[14];
}

// Build canonical tables from code lengths lens[0..n) (global scratch).  kind: 0 = code
// lengths (CODES), 1 = lit/len (LENS), 2 = distances (DISTS).  Returns false on zlib's
// "invalid ... set" conditions.
template <typename SymT>
__device__ __forceinline__ bool huff_build(const uint8_t* __restrict__ lens, int n, SymT* __restrict__ syms,
                           Huff& h, int kind) {
  uint32_t cnt[16], nhi[16];
#pragma unroll
  for (int L = 0; L < 16; ++L) cnt[L] = nhi[L] = 0;
  for (int s = 0; s < n; ++s) {
    const uint32_t len = lens[s];
    const uint32_t h = (kind == 1 && s >= 256) ? 1u : 0u;
#pragma unroll
    for (int L = 1; L < 16; ++L) {
      cnt[L] += (len == (uint32_t)L) ? 1u : 0u;
      nhi[L] += (len == (uint32_t)L) ? h : 0u;
    }
  }
  uint32_t maxl = 0;
#pragma unroll
  for (int L = 1; L < 16; ++L) maxl = cnt[L] ? (uint32_t)L : maxl;
  h.empty = (maxl == 0);
  if (maxl != 0) {
    int32_t left = 1;
    bool over = false;
#pragma unroll
    for (int L = 1; L < 16; ++L) {
      left = 2 * left - (int32_t)cnt[L];
      over |= left < 0;
    }
    if (over) return false;
    if (left > 0 && (kind == 0 || maxl != 1)) return false;  // incomplete set
  }
  uint32_t code = 0, base = 0;
  uint32_t next[16];
  int32_t prev_off = 0;
#pragma unroll
  for (int L = 1; L < 16; ++L) {
    h.lim[L - 1] = (code + cnt[L]) << (15 - L);
    h.hlim[L - 1] = (code + cnt[L] - nhi[L]) << (15 - L);
    const int32_t off = (int32_t)base - (int32_t)code;
    h.doff[L - 1] = off - prev_off;
    prev_off = off;
    next[L] = base;
    base += cnt[L];
    code = (code + cnt[L]) << 1;
  }
  if (maxl == 0) {
#pragma unroll
    for (int L = 0; L < 15; ++L) h.lim[L] = h.hlim[L] = 0;
  }
  for (int s = 0; s < n; ++s) {
    const uint32_t len = lens[s];
    if (len) {
      uint32_t pos = 0;
#pragma unroll
      for (int L = 1; L < 16; ++L) {
        const bool eq = (len == (uint32_t)L);
        pos = eq ? next[L] : pos;
        next[L] += eq ? 1u : 0u;
      }
      syms[pos] = (SymT)s;
    }
  }
  return true;
}

__device__ __forceinline__ void length_base(uint32_t sym, uint32_t& base, uint32_t& extra) {
  // sym in [257, 285]
  const uint32_t i = sym - 257u;
  if (i < 8u) { base = 3u + i; extra = 0u; }
  else if (i < 28u) { extra = (i - 4u) >> 2; base = ((4u + (i & 3u)) << extra) + 3u; }
  else { base = 258u; extra = 0u; }
}
__device__ __forceinline__ void dist_base(uint32_t d, uint32_t& base, uint32_t& extra) {
  // d in [0, 29]
  if (d < 4u) { base = d + 1u; extra = 0u; }
  else { extra = (d >> 1) - 1u; base = ((2u + (d & 1u)) << extra) + 1u; }
}

// Output sinks.  The decoder core below is the same for both; only how symbols land in
// memory differs.
//
// DirectSink: the whole block in a private buffer (guesser: BCIS needs the inflated block);
// LZ77 copies read the lane's own output.
struct DirectSink {
  uint8_t* out;
  __device__ __forceinline__ void literal(uint32_t op, uint32_t b) { out[op] = (uint8_t)b; }
  __device__ __forceinline__ void match(uint32_t op, uint32_t n, uint32_t dist) {
    // all sources lie in [op-dist, op): copy with period dist
    const uint8_t* src = out + (op - dist);
    uint8_t* dst = out + op;
    if (dist >= n) {
      uint32_t k = 0;
      for (; k + 4u <= n; k += 4u) {
        const uint8_t a0 = src[k], a1 = src[k + 1], a2 = src[k + 2], a3 = src[k + 3];
        dst[k] = a0; dst[k + 1] = a1; dst[k + 2] = a2; dst[k + 3] = a3;
      }
      for (; k < n; ++k) dst[k] = src[k];
    } else {
      uint32_t j = 0;
      for (uint32_t k = 0; k < n; ++k) {
        dst[k] = src[j];
        j = (j + 1u == dist) ? 0u : j + 1u;
      }
    }
  }
  __device__ __forceinline__ void finish(uint32_t) {}
};

// Inflate one raw DEFLATE stream (cdata, nbytes) to exactly isize bytes through `sink`.
// syms_ll: 288 LDS slots, u16 (symbol) or u8 (symbol & 255; bit 8 from Huff.hlim, which halves
// the batched inflate's LDS so two waves fit per SIMD); syms_d: 32 u8 LDS slots; lens: 352 B
// global scratch.  Returns INF_OK / INF_SHORT / INF_DATA; *produced = bytes accounted.
template <typename Sink, typename LLT>
__device__ int32_t inflate_core(const uint8_t* __restrict__ cdata, uint32_t nbytes, uint32_t isize,
                                LLT* __restrict__ syms_ll, uint8_t* __restrict__ syms_d,
                                uint8_t* __restrict__ lens, Sink& sink, uint32_t* produced) {
  BitIn br;
  br_init(br, cdata, nbytes);
  uint32_t op = 0;  // output position
  Huff hl, hd;
  bool last = false;
  int32_t rc = INF_OK;
  for (;;) {
    if (last) break;  // stream end
    br_refill(br);
    if (br_avail(br) < 3u) goto leave;
    last = (br.bb & 1u) != 0;
    const uint32_t type = (uint32_t)(br.bb >> 1) & 3u;
    br_drop(br, 3);
    if (type == 0u) {
      // stored: byte align, LEN/NLEN
      const uint32_t pad = (8u - (br.consumed & 7u)) & 7u;
      br_drop(br, pad);
      br_refill(br);
      if (br_avail(br) < 32u) goto leave;
      const uint32_t w = (uint32_t)br.bb;
      if ((w & 0xffffu) != ((w >> 16) ^ 0xffffu)) { rc = INF_DATA; goto done; }
      br_drop(br, 32);
      uint32_t len = w & 0xffffu;
      for (; len; --len) {
        if (op == isize) goto leave;
        br_refill(br);
        if (br_avail(br) < 8u) goto leave;
        sink.literal(op++, (uint32_t)br.bb & 0xffu);
        br_drop(br, 8);
      }
      continue;
    } else if (type == 1u) {
      // fixed Huffman code
      for (int s = 0; s < 288; ++s)
        lens[s] = (uint8_t)(s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8);
      for (int s = 0; s < 32; ++s) lens[288 + s] = 5;
      huff_build<LLT>(lens, 288, syms_ll, hl, 1);
      huff_build<uint8_t>(lens + 288, 32, syms_d, hd, 2);
    } else if (type == 2u) {
      br_refill(br);
      if (br_avail(br) < 14u) goto leave;
      const uint32_t nlen = ((uint32_t)br.bb & 31u) + 257u;
      const uint32_t ndist = ((uint32_t)(br.bb >> 5) & 31u) + 1u;
      const uint32_t ncode = ((uint32_t)(br.bb >> 10) & 15u) + 4u;
      br_drop(br, 14);
      if (nlen > 286u || ndist > 30u) { rc = INF_DATA; goto done; }
      // RFC 1951 code-length order 16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15
      // packed 5 bits per entry (a private array would be dynamically indexed -> scratch)
      const uint64_t ord_lo = 0x022caa324e804a30ULL, ord_hi = 0x00000003c2e1346cULL;
      for (int i = 0; i < 19; ++i) lens[i] = 0;
      for (uint32_t i = 0; i < ncode; ++i) {
        br_refill(br);
        if (br_avail(br) < 3u) goto leave;
        const uint32_t o = (uint32_t)((i < 12u ? ord_lo >> (5u * i) : ord_hi >> (5u * (i - 12u))) & 31u);
        lens[o] = (uint8_t)(br.bb & 7u);
        br_drop(br, 3);
      }
      Huff hc;
      if (!huff_build<LLT>(lens, 19, syms_ll, hc, 0)) { rc = INF_DATA; goto done; }
      // literal/length + distance code lengths (stored after the 19 CL lengths)
      uint8_t* ll = lens + 19;
      const uint32_t total = nlen + ndist;
      uint32_t have = 0;
      while (have < total) {
        br_refill(br);
        uint32_t L, sym;
        if (hc.empty) {
          L = 1;
          sym = 0;
          if (br_avail(br) < 1u) goto leave;
        } else {
          int32_t idx;
          const uint32_t v = br_rev15(br);
          huff_lookup(hc, v, L, idx);  // CODES sets are complete
          if (L > br_avail(br)) goto leave;
          sym = syms_ll[idx];
        }
        if (sym < 16u) {
          br_drop(br, L);
          ll[have++] = (uint8_t)sym;
          continue;
        }
        uint32_t xb = sym == 16u ? 2u : sym == 17u ? 3u : 7u;
        if (L + xb > br_avail(br)) goto leave;
        br_drop(br, L);
        uint32_t rep;
        uint8_t v8 = 0;
        if (sym == 16u) {
          if (have == 0) { rc = INF_DATA; goto done; }
          v8 = ll[have - 1];
          rep = 3u + br_peek(br, 2);
        } else if (sym == 17u) {
          rep = 3u + br_peek(br, 3);
        } else {
          rep = 11u + br_peek(br, 7);
        }
        br_drop(br, xb);
        if (have + rep > total) { rc = INF_DATA; goto done; }
        for (uint32_t k = 0; k < rep; ++k) ll[have++] = v8;
      }
      if (ll[256] == 0) { rc = INF_DATA; goto done; }
      if (!huff_build<LLT>(ll, (int)nlen, syms_ll, hl, 1)) { rc = INF_DATA; goto done; }
      if (!huff_build<uint8_t>(ll + nlen, (int)ndist, syms_d, hd, 2)) { rc = INF_DATA; goto done; }
    } else {
      rc = INF_DATA;  // invalid block type
      goto done;
    }
    // ---- symbols of a Huffman-coded block
    for (;;) {
      br_refill(br);
      uint32_t L;
      int32_t idx;
      const uint32_t v = br_rev15(br);
      uint32_t hi = 0;
      const bool ok = sizeof(LLT) == 1 ? huff_lookup_hi(hl, v, L, idx, hi) : huff_lookup(hl, v, L, idx);
      if (!ok) {
        if (br_avail(br) >= 1u) { rc = INF_DATA; goto done; }
        goto leave;
      }
      if (L > br_avail(br)) goto leave;
      const uint32_t sym = (uint32_t)syms_ll[idx] | hi;
      br_drop(br, L);
      if (sym < 256u) {
        if (op == isize) goto leave;
        sink.literal(op++, sym);
        continue;
      }
      if (sym == 256u) break;  // end of block
      if (sym > 285u) { rc = INF_DATA; goto done; }
      uint32_t lbase, lext;
      length_base(sym, lbase, lext);
      if (lext > br_avail(br)) goto leave;
      const uint32_t mlen = lbase + br_peek(br, lext);
      br_drop(br, lext);
      br_refill(br);
      const uint32_t vd = br_rev15(br);
      const bool okd = huff_lookup(hd, vd, L, idx);
      if (!okd) {
        if (br_avail(br) >= 1u) { rc = INF_DATA; goto done; }
        goto leave;
      }
      if (L > br_avail(br)) goto leave;
      const uint32_t dsym = syms_d[idx];
      br_drop(br, L);
      if (dsym > 29u) { rc = INF_DATA; goto done; }
      uint32_t dbase, dext;
      dist_base(dsym, dbase, dext);
      if (dext > br_avail(br)) goto leave;
      const uint32_t dist = dbase + br_peek(br, dext);
      br_drop(br, dext);
      if (op == isize) goto leave;
      if (dist > op) { rc = INF_DATA; goto done; }
      uint32_t n = isize - op;
      n = mlen < n ? mlen : n;
      sink.match(op, n, dist);
      op += n;
      if (n < mlen) goto leave;
    }
  }
leave:
  rc = (op == isize) ? INF_OK : INF_SHORT;
done:
  sink.finish(op);
  *produced = op;
  return rc;
}

// Single-pass inflate into a private buffer (used by the guesser's BCIS emulation).
__device__ __forceinline__ int32_t inflate_raw(const uint8_t* __restrict__ cdata, uint32_t nbytes,
                                               uint8_t* __restrict__ out, uint32_t isize,
                                               uint16_t* __restrict__ syms_ll,
                                               uint8_t* __restrict__ syms_d,
                                               uint8_t* __restrict__ lens, uint32_t* produced) {
  DirectSink s{out};
  return inflate_core(cdata, nbytes, isize, syms_ll, syms_d, lens, s, produced);
}

}  // namespace hbam
