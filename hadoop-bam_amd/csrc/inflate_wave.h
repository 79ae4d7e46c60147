// inflate_wave.h — wave-per-block Huffman pass of the batched BGZF inflate (k_inflate_wave), gfx950.
//
// Same contract and output as k_inflate_tokens (inflate_tok.h; zlib 1.2.11 semantics through
// [htsjdk] BlockGunzipper.unzipBlock -> java.util.zip.Inflater): literals at their final ubuf
// offsets, a 3-byte (len-3, dist-1) descriptor at the start of every match hole, one bit per
// match start in the block's bitmap, the partial first / last 16-byte chunks in the block's edge
// slot.  k_edge_merge and k_resolve run unchanged after it.
//
// What differs is the split of the work.  k_inflate_tokens gives each lane its own block, so each
// lane needs private decode tables (320 B of LDS and 236 VGPRs per lane: 2 waves per SIMD, a
// 14-compare canonical lookup per code).  Here the 64 lanes of a wave decode ONE block:
//   * the block's tables are built once per DEFLATE block by the whole wave into LDS: a direct
//     lookup of the first R = 10 stream bits (lit/len) / 8 bits (distance), and for longer codes a
//     flat table indexed by the 15-bit left-justified code value above the root's range, so one
//     LDS read decodes any code (u16 entries: symbol | length << 9, 7 KiB per wave in all);
//   * the symbol region of a DEFLATE block is cut into 64 bit ranges; lane i starts decoding a few
//     hundred bits before its range (a Huffman-coded stream resynchronises within a few tokens:
//     tools/spec_sim.py measures median 6, p99 42 tokens on the bench's data) and counts the
//     output bytes of the tokens that START inside its range;
//   * the wave checks that each lane's first counted token is the previous lane's exit token
//     (the first token at or after the range end); a lane that was not yet in step re-decodes
//     from the true start until it meets one of the positions it recorded on its first run;
//   * an exclusive scan of the counts gives every lane its output offset, and a second decode of
//     the lane's range writes the tokens (16-byte chunk stores inside the lane's range, byte
//     stores for chunks it shares with a neighbour, bitmap windows it shares zeroed first and
//     or-ed atomically).
// Any block this path does not cover exactly — a stored block, a code zlib would reject or that
// is incomplete, tables larger than the LDS budget, a stream that ends early or produces another
// length than ISIZE, a distance too far back — is left untouched except for writes inside its
// own output range and goes to a retry list that k_inflate_tokens then decodes with its full
// zlib error semantics.  So every block's result is what the lane-per-block pass gives.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "inflate_tok.h"

namespace hbam {

constexpr uint32_t WV_R = 10;     // lit/len root bits
constexpr uint32_t WV_DR = 8;     // distance root bits
constexpr uint32_t WV_TBL = 3072; // u16 table entries per wave: lit/len root + long, distance root + long
constexpr uint32_t WV_WARM = 256; // bits a lane decodes before its range to fall into step
// waves per SIMD asked of the register allocator (96 VGPRs, no spills; 4: 19.0 ms, 5: 18.2 ms at 2 GB)
constexpr uint32_t WV_WAVES = 5;
constexpr uint32_t WV_MINSEG = 512;   // bits per lane range at least
constexpr uint32_t WV_STAGE = 128;    // stream words staged in LDS for the header decode
constexpr uint32_t WV_TOK_BITS = 64;  // one iteration: 15 + 15 + 5 + 15 + 13 bits

#ifdef HBAM_WV_PROF
// Profiling build only (HBAM_WV_STATS prints them): wave cycles per phase summed over blocks,
// [0] header + code-length code, [1] lit/len + distance tables, [2] count pass, [3] in-step
// fixes, [4] offsets + window zeroing, [5] write pass, [6] fix rounds, [7] DEFLATE blocks
__device__ unsigned long long g_wvprof[8];
#define WV_T(i)                                                    \
  do {                                                             \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();              \
    if (threadIdx.x == 0) atomicAdd(&g_wvprof[i], t_ - wv_t0);     \
    wv_t0 = t_;                                                    \
  } while (0)
#define WV_N(i, n) \
  do { if (threadIdx.x == 0) atomicAdd(&g_wvprof[i], (unsigned long long)(n)); } while (0)
#else
#define WV_T(i) \
  do {          \
  } while (0)
#define WV_N(i, n) \
  do {             \
  } while (0)
#endif

struct WvLds {
  uint16_t tab[WV_TBL];  // lit/len root | lit/len long | distance root | distance long
  union {
    struct {
      uint8_t lens[320];  // code lengths: lit/len at [0, nlen), distance at [288, 288 + ndist)
      uint16_t clsorted[20];
      union {
        uint32_t stage[WV_STAGE + 4];  // header decode: stream words [w0, w0 + WV_STAGE + 4)
        uint16_t sorted[320];          // table build: symbols in canonical order
      } u;
    } b;
    uint8_t ring[64 * 32];  // write pass: two 16-byte output chunks per lane
  } v;
};

__device__ __forceinline__ uint32_t wv_uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint32_t wv_rank(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Canonical decode tables for the n code lengths at lens[] (wave-cooperative).  troot: 2^R
// entries indexed by the next R stream bits; tlong: one entry per 15-bit left-justified code value
// >= limR (codes longer than R).  Entry = symbol | length << 9, 0 = no code.  False for an
// over-subscribed or incomplete set (zlib rejects both, except a single-code distance set, which
// is left to the lane-per-block pass too) or when tlong would exceed long_cap entries.
__device__ bool wv_build(const uint8_t* lens, uint32_t n, uint16_t* sorted, uint16_t* troot, uint32_t R,
                         uint16_t* tlong, uint32_t long_cap, uint32_t& limR, uint32_t& nlong) {
  const uint32_t lane = threadIdx.x;
  uint32_t cnt[16];
#pragma unroll
  for (int l = 0; l < 16; ++l) cnt[l] = 0;
  for (uint32_t k = 0; k < n; k += 64) {
    const uint32_t s = k + lane;
    const uint32_t len = s < n ? lens[s] : 0u;
#pragma unroll
    for (int l = 1; l < 16; ++l) cnt[l] += (uint32_t)__popcll(__ballot(len == (uint32_t)l));
  }
  int32_t left = 1;
  bool bad = false;
#pragma unroll
  for (int l = 1; l < 16; ++l) {
    left = 2 * left - (int32_t)cnt[l];
    bad |= left < 0;
  }
  if (bad || left != 0) return false;
  Huff h;
  uint32_t code = 0, base = 0, next[16];
  int32_t prev = 0;
#pragma unroll
  for (int l = 1; l < 16; ++l) {
    h.lim[l - 1] = (code + cnt[l]) << (15 - l);
    h.hlim[l - 1] = 0;
    const int32_t off = (int32_t)base - (int32_t)code;
    h.doff[l - 1] = off - prev;
    prev = off;
    next[l] = base;
    base += cnt[l];
    code = (code + cnt[l]) << 1;
  }
  for (uint32_t k = 0; k < n; k += 64) {
    const uint32_t s = k + lane;
    const uint32_t len = s < n ? lens[s] : 0u;
    uint32_t pos = 0;
#pragma unroll
    for (int l = 1; l < 16; ++l) {
      const uint64_t m = __ballot(len == (uint32_t)l);
      pos = len == (uint32_t)l ? next[l] + wv_rank(m) : pos;
      next[l] += (uint32_t)__popcll(m);
    }
    if (len) sorted[pos] = (uint16_t)s;
  }
  __syncthreads();
  limR = h.lim[R - 1];
  nlong = 32768u - limR;
  if (nlong > long_cap) return false;
  HuffP hp;
  huffp_make(h, hp);
  for (uint32_t x = lane; x < (1u << R); x += 64) {
    const uint32_t v = __builtin_bitreverse32(x) >> 17;
    uint32_t L, idx, hi;
    const bool ok = huffp_lookup<false>(hp, v, L, idx, hi);
    troot[x] = (ok && L <= R) ? (uint16_t)(sorted[idx] | L << 9) : (uint16_t)0;
  }
  for (uint32_t j = lane; j < nlong; j += 64) {
    uint32_t L, idx, hi;
    const bool ok = huffp_lookup<false>(hp, limR + j, L, idx, hi);
    tlong[j] = ok ? (uint16_t)(sorted[idx] | L << 9) : (uint16_t)0;
  }
  __syncthreads();
  return true;
}

// uniform bit reader over stream words staged in LDS (the DEFLATE block headers)
struct WvHdr {
  const uint32_t* cw;  // 4-aligned stream base
  uint32_t wend;       // words that may be read (stream + BGZF footer)
  uint32_t w0;         // first staged word
  uint64_t bb;
  uint32_t bc, wn;     // valid bits in bb, next word to merge
};
__device__ __forceinline__ void wv_stage(WvLds& S, WvHdr& h, uint32_t w0) {
  __syncthreads();
  h.w0 = w0;
  for (uint32_t k = threadIdx.x; k < WV_STAGE + 4; k += 64) {
    const uint32_t w = w0 + k;
    S.v.b.u.stage[k] = w < h.wend ? h.cw[w] : 0u;
  }
  __syncthreads();
}
__device__ __forceinline__ uint32_t wv_word(WvLds& S, WvHdr& h, uint32_t w) {
  if (w < h.w0 || w >= h.w0 + WV_STAGE) wv_stage(S, h, w);
  return wv_uni(S.v.b.u.stage[w - h.w0]);
}
__device__ __forceinline__ void wv_hdr_at(WvLds& S, WvHdr& h, uint32_t q) {
  h.wn = q >> 5;
  h.bb = (uint64_t)(wv_word(S, h, h.wn) >> (q & 31u));
  h.bc = 32u - (q & 31u);
  ++h.wn;
}
__device__ __forceinline__ void wv_hdr_fill(WvLds& S, WvHdr& h) {  // >= 33 bits
  if (h.bc <= 32u) {
    h.bb |= (uint64_t)wv_word(S, h, h.wn) << h.bc;
    h.bc += 32u;
    ++h.wn;
  }
}
__device__ __forceinline__ void wv_hdr_drop(WvHdr& h, uint32_t n) {
  h.bb >>= n;
  h.bc -= n;
}
__device__ __forceinline__ uint32_t wv_hdr_pos(const WvHdr& h) { return h.wn * 32u - h.bc; }

// Header of the DEFLATE block at word-bit q: code lengths -> tables.  Uniform; false = leave the
// block to the lane-per-block pass.
struct WvTab {
  uint32_t llim, llong, droot, dlim, dlong;
};
__device__ bool wv_header(WvLds& S, WvHdr& h, uint32_t& q, uint32_t E, bool& bfinal, WvTab& t, uint64_t& wv_t0) {
  const uint32_t lane = threadIdx.x;
  wv_hdr_at(S, h, q);
  wv_hdr_fill(S, h);
  bfinal = (h.bb & 1u) != 0;
  const uint32_t type = (uint32_t)(h.bb >> 1) & 3u;
  wv_hdr_drop(h, 3);
  uint32_t nlen, ndist;
  if (type == 1u) {
    for (uint32_t s = lane; s < 320u; s += 64)
      S.v.b.lens[s] = (uint8_t)(s < 144u ? 8u : s < 256u ? 9u : s < 280u ? 7u : s < 288u ? 8u : 5u);
    nlen = 288;
    ndist = 32;
    __syncthreads();
  } else if (type == 2u) {
    wv_hdr_fill(S, h);
    nlen = ((uint32_t)h.bb & 31u) + 257u;
    ndist = ((uint32_t)(h.bb >> 5) & 31u) + 1u;
    const uint32_t ncode = ((uint32_t)(h.bb >> 10) & 15u) + 4u;
    wv_hdr_drop(h, 14);
    if (nlen > 286u || ndist > 30u) return false;
    // code-length code lengths, 3 bits each in RFC 1951 order; lane s < 19 takes symbol s's
    // (its position in the order: inverse of 16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15)
    const uint32_t s = lane;
    const uint64_t inv_lo = 0x0520c429d2b6be23ULL, inv_hi = 0x820941ccULL;  // 5 bits per symbol
    const uint32_t j = s < 12u ? (uint32_t)(inv_lo >> (5u * s)) & 31u
                               : s < 19u ? (uint32_t)(inv_hi >> (5u * (s - 12u))) & 31u : 31u;
    wv_hdr_fill(S, h);
    const uint32_t na = ncode < 10u ? ncode : 10u;
    uint32_t len = (j < na) ? (uint32_t)(h.bb >> (3u * j)) & 7u : 0u;
    wv_hdr_drop(h, 3u * na);
    wv_hdr_fill(S, h);
    if (j >= 10u && j < ncode && j < 19u) len = (uint32_t)(h.bb >> (3u * (j - 10u))) & 7u;
    wv_hdr_drop(h, 3u * (ncode - na));
    if (s < 19u) S.v.b.lens[s] = (uint8_t)len;
    __syncthreads();
    uint32_t clim, cnl;
    if (!wv_build(S.v.b.lens, 19, S.v.b.clsorted, S.tab, 7, S.tab + 128, 0, clim, cnl)) return false;
    // lit/len + distance code lengths (run-length coded; a run may cross from one to the other),
    // decoded 64 bit positions at a time: every lane decodes the code-length symbol that would
    // start at its bit, a uniform walk over the lanes (v_readlane) picks out the true ones, and
    // scans give each its place and the value a code 16 repeats.  Only nonzero lengths are
    // stored (the arrays are zeroed first): runs of zeros (17, 18) cost no writes.
    for (uint32_t i2 = lane; i2 < 320u; i2 += 64) S.v.b.lens[i2] = 0;
    __syncthreads();
    const uint32_t total = nlen + ndist;
    uint32_t have = 0, carry = ~0u, qq = wv_hdr_pos(h);
    while (have < total) {
      const uint32_t wb = qq >> 5;
      if (wb < h.w0 || wb + 4u > h.w0 + WV_STAGE) wv_stage(S, h, wb);
      const uint32_t P = qq + lane, w = (P >> 5) - h.w0, sh = P & 31u;
      const uint64_t two = (uint64_t)S.v.b.u.stage[w] | (uint64_t)S.v.b.u.stage[w + 1] << 32;
      const uint32_t bits = (uint32_t)(two >> sh);
      const uint32_t e = S.tab[bits & 127u];
      const uint32_t L = e >> 9, sym = e & 511u;
      const uint32_t xb = sym == 16u ? 2u : sym == 17u ? 3u : sym == 18u ? 7u : 0u;
      const uint32_t xv = (bits >> L) & ((1u << xb) - 1u);
      const uint32_t adv = L + xb;
      const uint32_t rep = sym < 16u ? 1u : sym == 18u ? 11u + xv : 3u + xv;
      uint64_t vis = 0;
      uint32_t pp = 0, hv = have;
      while (pp < 64u && hv < total) {
        vis |= 1ull << pp;
        hv += (uint32_t)__builtin_amdgcn_readlane((int)rep, (int)pp);
        pp += (uint32_t)__builtin_amdgcn_readlane((int)adv, (int)pp);
      }
      if (hv > total) return false;  // a run past the last length (zlib: invalid bit length repeat)
      const bool me = ((vis >> lane) & 1u) != 0u;
      const uint32_t r = me ? rep : 0u;
      uint32_t incl = r, km = (me && sym != 16u) ? lane + 1u : 0u;
#pragma unroll
      for (uint32_t dlt = 1; dlt < 64u; dlt <<= 1) {
        const uint32_t y = __shfl_up(incl, dlt), z = __shfl_up(km, dlt);
        incl += lane >= dlt ? y : 0u;
        km = (lane >= dlt && z > km) ? z : km;
      }
      const uint32_t own = sym < 16u ? sym : 0u;
      const uint32_t pv = __shfl(own, km ? km - 1u : 0u);
      const uint32_t val = sym == 16u ? (km ? pv : carry) : own;
      if (__any(me && sym == 16u && val == ~0u)) return false;  // a repeat with nothing before it
      const uint32_t hb = have + incl - r;
      if (me && val != 0u)
        for (uint32_t k = 0; k < rep; ++k) {
          const uint32_t i2 = hb + k;
          S.v.b.lens[i2 < nlen ? i2 : 288u + (i2 - nlen)] = (uint8_t)val;
        }
      carry = wv_uni(__shfl(val, 63u - (uint32_t)__builtin_clzll(vis)));
      have = hv;
      qq += pp;
    }
    __syncthreads();
    if (wv_uni(S.v.b.lens[256]) == 0u) return false;
    wv_hdr_at(S, h, qq);
  } else {
    return false;  // stored (or invalid) block: the lane-per-block pass
  }
  q = wv_hdr_pos(h);
  WV_T(0);
  if (q > E) return false;
  h.w0 = 0xffffffffu - WV_STAGE;  // the table build reuses the staging area
  uint32_t nll, nd;
  if (!wv_build(S.v.b.lens, nlen, S.v.b.u.sorted, S.tab, WV_R, S.tab + (1u << WV_R), WV_TBL - (1u << WV_R) - (1u << WV_DR),
                t.llim, nll))
    return false;
  t.llong = 1u << WV_R;
  t.droot = t.llong + nll;
  t.dlong = t.droot + (1u << WV_DR);
  if (!wv_build(S.v.b.lens + 288, ndist, S.v.b.u.sorted + 288, S.tab + t.droot, WV_DR, S.tab + t.dlong, WV_TBL - t.dlong,
                t.dlim, nd))
    return false;
  return true;
}

// ---- lane reader: the input epochs of inflate_tok.h's EIn (two 16-byte banks + one quad in
// flight, merged / requested by every lane at the same iteration); the decode loops are per-lane
// do-while loops with a scalar epoch branch, as the lane pass's symbol loop (a wave-uniform
// `while (__any(...))` loop made the compiler copy the reader's registers, and wait on the quad in
// flight, at every iteration).
__device__ __forceinline__ u32x4_t wv_load(const uint4* p) {
  return ein_load(p);
}
struct WvBits {
  uint64_t bb;
  uint32_t bc, rd, nv, pos;  // valid bits, next bank dword, dwords left in the banks, word-bit position
};
struct WvIn {
  const uint4* fp;
  const uint4* fend;
  const uint4* safe;
  uint4 q0, q1;
  u32x4_t t;
  WvBits s;
};
__device__ __forceinline__ uint32_t wv_sel(const WvIn& in, uint32_t i) {
  const bool h = (i & 4u) != 0u, z = (i & 2u) != 0u;
  const uint32_t x = h ? in.q1.x : in.q0.x, y = h ? in.q1.y : in.q0.y;
  const uint32_t zz = h ? in.q1.z : in.q0.z, w = h ? in.q1.w : in.q0.w;
  const uint32_t a = z ? zz : x, b = z ? w : y;
  return (i & 1u) ? b : a;
}
// reader at word-bit p of the stream (4-aligned base cw) whose bits end at word-bit E
__device__ __forceinline__ void wv_in_at(WvIn& in, const uint32_t* cw, uint32_t p, uint32_t E) {
  const uint8_t* c8 = (const uint8_t*)cw;
  const uint32_t b0 = p >> 3, eb = (E + 7u) >> 3;  // p may lie a token past E on a path out of step
  const uint8_t* q = c8 + b0;
  const uintptr_t a = (uintptr_t)q & 15u;
  const uint4* base = (const uint4*)(q - a);
  in.fend = (const uint4*)(((uintptr_t)(c8 + (b0 < eb ? eb : b0)) + 15u) & ~(uintptr_t)15u);
  in.safe = base;
  in.q0 = base[0];
  in.q1 = base[1];
  in.fp = base + 2 < in.fend ? base + 2 : in.fend;
  in.t = wv_load(in.fp < in.fend ? in.fp : in.safe);
  const uint32_t r = (uint32_t)(a >> 2), sh = 8u * (uint32_t)(a & 3u) + (p & 7u);
  in.s.bb = (uint64_t)(wv_sel(in, r) >> sh);
  in.s.bc = 32u - sh;
  in.s.rd = r + 1u;
  in.s.nv = 8u - in.s.rd;
  in.s.pos = p;
}
__device__ __forceinline__ void wv_epoch(WvIn& in) {
  if (in.fp < in.fend && in.s.nv <= 4u) {
    const bool hi = (((in.s.rd + in.s.nv) & 7u) >> 2) != 0u;
    const u32x4_t t = in.t;
    in.q0.x = hi ? in.q0.x : t[0];
    in.q0.y = hi ? in.q0.y : t[1];
    in.q0.z = hi ? in.q0.z : t[2];
    in.q0.w = hi ? in.q0.w : t[3];
    in.q1.x = hi ? t[0] : in.q1.x;
    in.q1.y = hi ? t[1] : in.q1.y;
    in.q1.z = hi ? t[2] : in.q1.z;
    in.q1.w = hi ? t[3] : in.q1.w;
    in.s.nv += 4u;
    ++in.fp;
  }
  in.t = wv_load(in.fp < in.fend ? in.fp : in.safe);
}
__device__ __forceinline__ bool wv_short(const WvIn& in, uint32_t need) {
  return in.s.bc + 32u * in.s.nv < need && in.fp < in.fend;
}
__device__ __forceinline__ void wv_fill(const WvIn& in, WvBits& s) {
  const bool m = s.bc <= 32u && s.nv != 0u;
  const uint64_t w = (uint64_t)wv_sel(in, s.rd) << (s.bc & 63u);
  s.bb = m ? s.bb | w : s.bb;
  s.bc = m ? s.bc + 32u : s.bc;
  s.rd = m ? (s.rd + 1u) & 7u : s.rd;
  s.nv = m ? s.nv - 1u : s.nv;
}
__device__ __forceinline__ void wv_drop(WvBits& s, uint32_t n) {
  s.bb >>= n;
  s.bc -= n;
  s.pos += n;
}
__device__ __forceinline__ uint32_t wv_peek(const WvBits& s, uint32_t n) { return (uint32_t)s.bb & ((1u << n) - 1u); }

// One iteration of a decode loop: token A at s.pos, and when A is a literal whose successor
// starts before `lim`, token B too (60 % of tokens are literals: 1.6 tokens per iteration, as
// tok_fast_spec in inflate_tok.h).  One match path per iteration, fed by A or by B.  Kinds:
// 0 literal, 1 match, 2 end of block, 3 invalid code; kB = 4 when B is not taken.  a1 / a2: the
// literal bytes; len / dist: the match; p2 = B's start.  Table indices stay inside the tables
// whatever the bits, so lanes past their range decode garbage harmlessly.
struct WvIt {
  uint32_t kA, kB, a1, a2, len, dist, p2;
};
__device__ __forceinline__ void wv_tok2(const WvIn& in, WvBits& s, const uint16_t* __restrict__ tab,
                                        const WvTab& t, uint32_t lim, WvIt& o) {
  wv_fill(in, s);
  uint32_t v = (uint32_t)s.bb;
  uint32_t v15 = __builtin_bitreverse32(v) >> 17;
  const uint32_t e1 = tab[v15 >= t.llim ? t.llong + (v15 - t.llim) : (v & ((1u << WV_R) - 1u))];
  const uint32_t L1 = e1 >> 9, sym1 = e1 & 511u;
  wv_drop(s, L1);
  o.p2 = s.pos;
  wv_fill(in, s);
  v = (uint32_t)s.bb;
  v15 = __builtin_bitreverse32(v) >> 17;
  const uint32_t e2 = tab[v15 >= t.llim ? t.llong + (v15 - t.llim) : (v & ((1u << WV_R) - 1u))];
  const uint32_t L2 = e2 >> 9, sym2 = e2 & 511u;
  const bool lit1 = L1 != 0u && sym1 < 256u;
  const bool useB = lit1 && o.p2 < lim;
  wv_drop(s, useB ? L2 : 0u);
  const uint32_t m = useB ? sym2 : sym1;
  const bool mok = useB ? L2 != 0u : L1 != 0u;
  const bool ism = (useB || !lit1) && mok && m > 256u && m <= 285u;
  uint32_t lb, le;
  length_base(ism ? m : 257u, lb, le);
  le = ism ? le : 0u;
  wv_fill(in, s);
  o.len = lb + wv_peek(s, le);
  wv_drop(s, le);
  v = (uint32_t)s.bb;
  v15 = __builtin_bitreverse32(v) >> 17;
  const uint32_t e3 = tab[v15 >= t.dlim ? t.dlong + (v15 - t.dlim) : t.droot + (v & ((1u << WV_DR) - 1u))];
  const uint32_t L3 = ism ? e3 >> 9 : 0u, ds = e3 & 511u;
  wv_drop(s, L3);
  const bool dok = L3 != 0u && ds <= 29u;
  uint32_t db, de;
  dist_base(dok ? ds : 0u, db, de);
  de = (ism && dok) ? de : 0u;
  o.dist = db + wv_peek(s, de);
  wv_drop(s, de);
  const uint32_t km = !mok || m > 285u ? 3u : m < 256u ? 0u : m == 256u ? 2u : dok ? 1u : 3u;
  o.kA = lit1 ? 0u : km;
  o.kB = useB ? km : 4u;
  o.a1 = sym1;
  o.a2 = sym2;
}

// Output of one lane's range [olo, ohi) (block-relative).  Bytes go to a two-chunk ring of the
// lane in LDS (ring[(soff + op) & 31]); when the lane moves on, a finished 16-byte chunk it holds
// alone is one store, one it shares with a neighbour lane (or the block's first / last partial
// chunk, which goes to the edge slot) is written bytewise.  Hole bytes of a chunk keep whatever
// the ring held: k_resolve overwrites every hole.  Bitmap windows: registers; windows the lane
// holds alone are one store, shared ones (zeroed before the pass) are or-ed atomically.
struct WSink {
  uint8_t* cbase;  // 16-aligned address of chunk 0
  uint8_t* edge;
  uint32_t* bm;
  uint8_t* ring;   // this lane's 32 bytes
  uint32_t soff, iend, isize;
  uint32_t olo, ohi;
  uint32_t curc;   // chunk of the last byte written (~0u: none)
  bool sp;         // the last descriptor ran into chunk curc + 1
  uint32_t bwin, w0, w1, w2, w3;

  __device__ __forceinline__ void flushc(uint32_t c) {
    const uint32_t r0 = c << 4;
    const bool inblk = r0 >= soff && r0 + 16u <= iend;
    const bool excl = r0 >= soff + olo && r0 + 16u <= soff + ohi;
    const uint8_t* src = ring + ((c & 1u) << 4);
    if (inblk && excl) {
      st_out((uint4*)(cbase + r0), *(const uint4*)src);
    } else {
      uint8_t* dst = inblk ? cbase + r0 : edge + (r0 < soff ? 0u : 16u);
      const uint32_t a = r0 > soff + olo ? r0 : soff + olo;
      const uint32_t z = r0 + 16u < soff + ohi ? r0 + 16u : soff + ohi;
      for (uint32_t r = a; r < z; ++r) dst[r & 15u] = src[r & 15u];
    }
  }
  __device__ __forceinline__ void to_chunk(uint32_t c) {
    if (c != curc) {
      if (curc != ~0u) {
        flushc(curc);
        if (sp && c != curc + 1u) flushc(curc + 1u);
      }
      curc = c;
      sp = false;
    }
  }
  __device__ __forceinline__ void lit(uint32_t op, uint32_t b) {
    const uint32_t r = soff + op;
    to_chunk(r >> 4);
    ring[r & 31u] = (uint8_t)b;
  }
  __device__ __forceinline__ void desc(uint32_t op, uint32_t v) {  // 3 bytes
    const uint32_t r = soff + op;
    to_chunk(r >> 4);
    ring[r & 31u] = (uint8_t)v;
    ring[(r + 1u) & 31u] = (uint8_t)(v >> 8);
    ring[(r + 2u) & 31u] = (uint8_t)(v >> 16);
    sp = (r & 15u) > 13u;
  }
  __device__ __forceinline__ bool win_excl(uint32_t W) const {
    const uint32_t p0 = W << 7, p1 = (p0 + 128u < isize) ? p0 + 128u : isize;
    return p0 >= olo && p1 <= ohi;
  }
  __device__ __forceinline__ void win_flush() {
    uint32_t* p = bm + 4u * bwin;
    if (win_excl(bwin)) {
      st_out((uint4*)p, make_uint4(w0, w1, w2, w3));
    } else {
      if (w0) atomicOr(p, w0);
      if (w1) atomicOr(p + 1, w1);
      if (w2) atomicOr(p + 2, w2);
      if (w3) atomicOr(p + 3, w3);
    }
  }
  __device__ __forceinline__ void win_to(uint32_t w) {
    while (bwin < w) {
      win_flush();
      w0 = w1 = w2 = w3 = 0;
      ++bwin;
    }
  }
  // match-start bit at op when m (the window switch is the only branch)
  __device__ __forceinline__ void mark(bool m, uint32_t op) {
    const uint32_t w = op >> 7;
    if (m && w != bwin) win_to(w);
    const uint32_t i = op & 127u, b = m ? 1u << (i & 31u) : 0u, q = i >> 5;
    w0 |= q == 0u ? b : 0u;
    w1 |= q == 1u ? b : 0u;
    w2 |= q == 2u ? b : 0u;
    w3 |= q == 3u ? b : 0u;
  }
  __device__ __forceinline__ void finish() {
    if (curc != ~0u) {
      flushc(curc);
      if (sp) flushc(curc + 1u);
    }
    win_to(((ohi - 1u) >> 7) + 1u);
  }
};

// Decode one BGZF block with the whole wave.  True: the block's output, bitmap and edge slot
// are written.  False: left to the lane-per-block pass (nothing outside the block's own output
// range, bitmap and edge slot was written).
__device__ bool inflate_wave_block(WvLds& S, const uint8_t* __restrict__ cdata, uint32_t nbytes, uint32_t isize,
                                   uint8_t* __restrict__ ubuf, uint64_t start, uint32_t* __restrict__ bm,
                                   uint8_t* __restrict__ edge) {
  const uint32_t lane = threadIdx.x;
  const uint32_t* cw = (const uint32_t*)((uintptr_t)cdata & ~(uintptr_t)3);
  const uint32_t boff = 8u * (uint32_t)((uintptr_t)cdata & 3u);
  const uint32_t E = boff + 8u * nbytes;  // word-bit end of the stream
  WvHdr h;
  h.cw = cw;
  h.wend = (E + 31u) / 32u + 2u;  // + the BGZF footer
  h.w0 = 0xffffffffu - WV_STAGE;
  uint32_t q = boff;
  uint32_t out = 0;
  bool bfinal = false;
  uint8_t* cbase = ubuf + (start & ~15ull);
  const uint32_t soff = (uint32_t)(start & 15u);
  uint32_t it = 0;  // epoch clock (uniform)
  uint64_t wv_t0 = __builtin_amdgcn_s_memtime();
  (void)wv_t0;
  for (uint32_t blkno = 0; !bfinal; ++blkno) {
    WvTab t;
    if (!wv_header(S, h, q, E, bfinal, t, wv_t0)) return false;
    WV_T(1);
    WV_N(7, 1);
    const uint32_t Sb = q;  // first symbol bit
    // ---- count pass
    uint32_t seg = (E - Sb + 63u) >> 6;
    seg = seg < WV_MINSEG ? WV_MINSEG : seg;
    const uint32_t lo = Sb + lane * seg;
    const uint32_t hi = lo + seg < E ? lo + seg : E;
    const bool has = lo < E;
    const uint32_t st = lane == 0 ? Sb : (lo > Sb + WV_WARM ? lo - WV_WARM : Sb);
    WvIn in;
    wv_in_at(in, cw, has ? st : Sb, E);
    // c counts output bytes from the lane's start (warm-up included); cf = c at the first
    // counted token f; checkpoints (cp, cc) = (position, c) at two later tokens
    uint32_t f = ~0u, cf = 0, x = ~0u, c = 0, nt = 0, fl = 0, eend = 0;
    uint32_t cp1 = ~0u, cc1 = 0, cp2 = ~0u, cc2 = 0;
    bool act = has;
    // per-lane loops as in inflate_tok.h (a lane leaves when done; the epoch branch is scalar
    // through readfirstlane: every active lane has the same clock)
    if (act) do {
      if ((wv_uni(++it) & (TOK_K - 1u)) == 0u) wv_epoch(in);
      if (!wv_short(in, WV_TOK_BITS)) {
        const uint32_t pos = in.s.pos;
        if (pos >= hi) {
          x = pos;
          act = false;
        } else {
          WvIt o;
          wv_tok2(in, in.s, S.tab, t, hi, o);
          // token A at pos
          bool first = f == ~0u && pos >= lo;
          f = first ? pos : f;
          cf = first ? c : cf;
          cp1 = nt == 40u ? pos : cp1;
          cc1 = nt == 40u ? c : cc1;
          cp2 = nt == 120u ? pos : cp2;
          cc2 = nt == 120u ? c : cc2;
          c += o.kA == 0u ? 1u : o.kA == 1u ? o.len : 0u;
          ++nt;
          // token B at p2
          const bool tb = o.kB != 4u;
          first = tb && f == ~0u && o.p2 >= lo;
          f = first ? o.p2 : f;
          cf = first ? c : cf;
          cp1 = (tb && nt == 40u) ? o.p2 : cp1;
          cc1 = (tb && nt == 40u) ? c : cc1;
          cp2 = (tb && nt == 120u) ? o.p2 : cp2;
          cc2 = (tb && nt == 120u) ? c : cc2;
          c += o.kB == 0u ? 1u : o.kB == 1u ? o.len : 0u;
          nt += tb ? 1u : 0u;
          const uint32_t ks = o.kA >= 2u ? o.kA : (o.kB >= 2u && o.kB != 4u) ? o.kB : 0u;
          if (ks) {
            fl = ks;
            eend = in.s.pos;
            act = false;
          }
        }
      }
    } while (act);
    WV_T(2);
    // ---- in-step check: lane i's first counted token must be lane i-1's exit token
    uint32_t e = 64;
    for (uint32_t round = 0;; ++round) {
      const uint32_t xp = __shfl_up(x, 1);
      const uint64_t em = __ballot(fl != 0u && f != ~0u);
      e = em ? (uint32_t)__builtin_ctzll(em) : 64u;
      const bool need = lane > 0u && lane <= e && f != xp;
      if (!__any(need)) break;
      if (round >= 64u) return false;
      WV_N(6, 1);
      // re-decode from the true start until a position of the first run is met (the lowest
      // lane out of step always has a valid start; a higher one may not yet)
      const bool fix = need && xp != ~0u;
      bool fx = fix;
      uint32_t c2 = 0;
      if (fix) wv_in_at(in, cw, xp, E);
      if (fx) do {
        if ((wv_uni(++it) & (TOK_K - 1u)) == 0u) wv_epoch(in);
        if (!wv_short(in, WV_TOK_BITS)) {
          const uint32_t pos = in.s.pos;
          if (pos >= hi) {
            x = pos;
            c = c2;
            fl = 0;
            fx = false;
          } else if (pos == f || pos == cp1 || pos == cp2) {
            c = c2 + (c - (pos == f ? cf : pos == cp1 ? cc1 : cc2));
            fx = false;
          } else {
            WvIt o;
            wv_tok2(in, in.s, S.tab, t, hi, o);
            if (o.kA >= 2u) {
              fl = o.kA;
              eend = in.s.pos;
              c = c2;
              fx = false;
            } else {
              c2 += o.kA == 0u ? 1u : o.len;
              if (o.kB != 4u) {
                if (o.p2 == f || o.p2 == cp1 || o.p2 == cp2) {  // in step from B on
                  c = c2 + (c - (o.p2 == f ? cf : o.p2 == cp1 ? cc1 : cc2));
                  fx = false;
                } else if (o.kB >= 2u) {
                  fl = o.kB;
                  eend = in.s.pos;
                  c = c2;
                  fx = false;
                } else {
                  c2 += o.kB == 0u ? 1u : o.len;
                }
              }
            }
          }
        }
      } while (fx);
      f = fix ? xp : f;
      cf = fix ? 0u : cf;
      cp1 = fix ? ~0u : cp1;
      cp2 = fix ? ~0u : cp2;
    }
    c -= cf;
    if (e == 64u) return false;                     // no end of block before the stream end
    if (wv_uni(__shfl(fl, e)) != 2u) return false;  // an invalid code (3) on the true path
    const uint32_t qn = wv_uni(__shfl(eend, e));
    if (qn > E) return false;
    WV_T(3);
    // ---- output offsets
    const uint32_t cc = lane <= e ? c : 0u;
    uint32_t incl = cc;
#pragma unroll
    for (uint32_t dlt = 1; dlt < 64u; dlt <<= 1) {
      const uint32_t y = __shfl_up(incl, dlt);
      incl += lane >= dlt ? y : 0u;
    }
    const uint32_t total = wv_uni(__shfl(incl, 63));
    if (out + total > isize) return false;
    if (bfinal && out + total != isize) return false;
    const uint32_t olo = out + incl - cc, ohi = olo + cc;
    // ---- write pass
    WSink sk;
    sk.cbase = cbase;
    sk.edge = edge;
    sk.bm = bm;
    sk.soff = soff;
    sk.iend = soff + isize;
    sk.isize = isize;
    sk.olo = olo;
    sk.ohi = ohi;
    sk.ring = S.v.ring + 32u * lane;
    sk.curc = ~0u;
    sk.sp = false;
    sk.bwin = olo >> 7;
    sk.w0 = sk.w1 = sk.w2 = sk.w3 = 0;
    const uint32_t skipw = (blkno > 0u && (out & 127u)) ? out >> 7 : ~0u;
    if (cc) {
      const uint32_t fw = olo >> 7, lw = (ohi - 1u) >> 7;
      if (!sk.win_excl(fw) && fw != skipw) st_out((uint4*)(bm + 4u * fw), make_uint4(0, 0, 0, 0));
      if (lw != fw && !sk.win_excl(lw) && lw != skipw) st_out((uint4*)(bm + 4u * lw), make_uint4(0, 0, 0, 0));
    }
    __builtin_amdgcn_s_waitcnt(0);
    WV_T(4);
    bool wa = cc != 0u;
    bool bad = false;
    uint32_t op = olo;
    if (wa) wv_in_at(in, cw, f, E);
    if (wa) do {
      if ((wv_uni(++it) & (TOK_K - 1u)) == 0u) wv_epoch(in);
      if (!wv_short(in, WV_TOK_BITS)) {
        if (in.s.pos >= hi) {
          wa = false;
        } else {
          WvIt o;
          wv_tok2(in, in.s, S.tab, t, hi, o);
          // A: literal or match; B (after a literal A): literal or match; one match at most
          const bool ma = o.kA == 1u, mb = o.kB == 1u;
          const uint32_t nA = o.kA == 0u ? 1u : ma ? o.len : 0u;
          const uint32_t nB = o.kB == 0u ? 1u : mb ? o.len : 0u;
          const bool stop = o.kA >= 2u || (o.kB >= 2u && o.kB != 4u);
          const bool eob = (o.kA == 2u) || (o.kA == 0u && o.kB == 2u);
          if (op + nA + nB > ohi || (stop && !eob)) {  // cannot happen on the counted path
            bad = true;
            wa = false;
          } else {
            if (o.kA == 0u) sk.lit(op, o.a1);
            if (o.kB == 0u) sk.lit(op + 1u, o.a2);
            const uint32_t om = ma ? op : op + 1u;
            const bool mm = ma || mb;
            bad = bad || (mm && o.dist > om);
            if (mm) sk.desc(om, (o.len - 3u) | (o.dist - 1u) << 8);
            sk.mark(mm, om);
            op += nA + nB;
            wa = !stop;
          }
        }
      }
    } while (wa);
    if (cc) sk.finish();
    WV_T(5);
    if (__any(bad)) return false;
    out += total;
    q = qn;
  }
  return out == isize;
}

}  // namespace hbam
