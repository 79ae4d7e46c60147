// inflate_par.h — phase 1 of the batched inflate, one workgroup of PI_NL lanes per BGZF block.
//
// Replaces the lane-per-block Huffman pass for well-formed blocks ([htsjdk]
// BlockGunzipper.unzipBlock -> JDK zlib Inflater; BAMRecordReader.java:133-143).  Output
// format is the TokenSink one (inflate_dev.h): literals at their final offsets in ubuf, a
// 3-byte descriptor (len-3, dist-1) in the first bytes of every match and a bit per match
// start in the block's bitmap, so k_resolve (resolve_dev.h) finishes the block unchanged.
//
// Parallel Huffman decode by self-synchronisation.  Per DEFLATE block the header is decoded
// once (wave-uniform) and its canonical codes are expanded into LDS lookup tables shared by
// the workgroup (12-bit lit/len root, 10-bit distance root; longer codes take a 2-4 compare
// canonical step).  The remaining bit stream [pos, T) is cut into PI_NL segments:
//   pass 1   every lane decodes its segment from the segment's first bit as if a token
//            started there, counting output bytes and recording the bit lengths of its first
//            PI_M tokens (u8 deltas) and its first PI_E end-of-block codes;
//   sync     lane i keeps decoding past its segment end until one of its token starts
//            coincides with a recorded token start of lane i+1: from there on both decodes
//            are the same (same tables, same state), so lane i+1's decode is true from that
//            point (Huffman codes self-synchronise within a few tokens);
//   plan     lane l is true from P_l (lane 0: the pass start; lane l: the point lane l-1
//            synchronised at).  The first lane whose true region holds an end-of-block code
//            ends the DEFLATE block; a lane that failed to synchronise ends the commit (the
//            next round restarts from where that lane stopped, so progress is guaranteed);
//            byte counts -> exclusive scan -> output offsets;
//   pass 2   committed lanes re-decode their true regions and emit.
// Everything the fast path does not handle exactly like zlib 1.2.11 (stored-length errors,
// incomplete or over-subscribed codes, invalid symbols or distances in a true region,
// output not ending exactly at ISIZE with the final block, input overrun, > PI_MAX_ROUNDS
// rounds) marks the block INF_RETRY; the lane-per-block inflate_core (zlib-exact contract)
// then redoes it from scratch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "inflate_dev.h"

namespace hbam {

constexpr uint32_t PI_NL = 128;          // lanes (segments) per block
constexpr uint32_t PI_WAVES = PI_NL / 64;
constexpr uint32_t PI_LL_ROOT = 12;
constexpr uint32_t PI_D_ROOT = 10;
constexpr uint32_t PI_M = 64;            // token starts recorded per lane (sync within M tokens:
                                         // 99.9 % of random starts on level-5 BAM data)
constexpr uint32_t PI_E = 2;             // end-of-block codes recorded per lane
constexpr uint32_t PI_MIN_SEG = 2048;    // bits per segment, at least (~200 tokens: sync needs up to ~70)
constexpr uint32_t PI_MAX_ROUNDS = 256;
constexpr int32_t INF_RETRY = 3;
constexpr uint32_t PI_NONE = 0xffffffffu;

struct PiShared {
  uint16_t ll[1u << PI_LL_ROOT];   // len | sym << 4 (len 0: longer code)
  uint16_t d[1u << PI_D_ROOT];
  uint16_t sll[288];               // symbols in canonical order (long codes)
  uint16_t sd[32];
  uint16_t codes[320];             // per symbol: bit-reversed canonical code
  uint16_t cl[128];                // code-length code table (7-bit root, complete)
  uint8_t lens[352];               // 19 CL lengths | HLIT + HDIST lengths
  uint32_t lim_ll[16], lim_d[16];  // lim[L] = (first_L + cnt_L) << (15 - L)
  int32_t off_ll[16], off_d[16];   // off[L] = (# shorter codes) - first_L
  uint32_t cnt[2][16];
  uint32_t bm[BITMAP_WORDS];       // match-start bitmap of the block
  uint8_t bdel[PI_NL * PI_M];      // bit length of each of the segment's first tokens
  uint32_t eob_s[PI_NL * PI_E], eob_e[PI_NL * PI_E], eob_c[PI_NL * PI_E];
  uint8_t nbnd[PI_NL], neob[PI_NL];
  uint32_t tot[PI_NL];             // pass-1 bytes (segment start -> pass-1 stop)
  uint32_t syn_pos[PI_NL];         // lane i: where it met lane i+1's decode (PI_NONE: did not)
  uint32_t syn_idx[PI_NL];         // lane i+1's token index at syn_pos[i]
  uint32_t syn_bytes[PI_NL];       // lane i's bytes from its segment start to syn_pos / stop
  uint32_t syn_stop[PI_NL];        // lane i: where its decode stopped (sync failure)
  uint32_t wsum[PI_WAVES];
  uint32_t u[8];                   // uniform plan values
};

// ---- bit reader over a raw DEFLATE stream, starting at an arbitrary bit ----
struct PBits {
  BitIn b;
  uint32_t pos;  // stream bit of bb's bit 0
};
__device__ __forceinline__ void pb_init(PBits& r, const uint8_t* cdata, uint32_t bit) {
  br_init(r.b, cdata + (bit >> 3), 1u << 20);
  r.pos = bit & ~7u;
  br_refill(r.b);
  const uint32_t k = bit & 7u;
  r.b.bb >>= k;
  r.b.bc -= k;
  r.pos = bit;
}
__device__ __forceinline__ void pb_drop(PBits& r, uint32_t n) {
  r.b.bb >>= n;
  r.b.bc -= n;
  r.pos += n;
}

// ---- one token.  kind: 0 literal (v = byte), 1 match (v = len, w = dist), 2 end of block,
// 3 invalid symbol.  Consumes its bits.
__device__ __forceinline__ uint32_t pi_long(const uint32_t* lim, const int32_t* off, const uint16_t* syms,
                                            uint32_t root, uint64_t bb, uint32_t& L) {
  const uint32_t v = __builtin_bitreverse32((uint32_t)bb) >> 17;
  uint32_t l = root + 1;
  for (uint32_t k = root + 1; k < 15; ++k) l += (v >= lim[k]) ? 1u : 0u;
  L = l;
  return syms[off[l] + (int32_t)(v >> (15u - l))];
}

__device__ __forceinline__ uint32_t pi_token(const PiShared& s, PBits& r, uint32_t& v, uint32_t& w) {
  br_refill(r.b);
  uint32_t e = s.ll[(uint32_t)r.b.bb & ((1u << PI_LL_ROOT) - 1)];
  uint32_t L = e & 15u, sym = e >> 4;
  if (L == 0) sym = pi_long(s.lim_ll, s.off_ll, s.sll, PI_LL_ROOT, r.b.bb, L);
  if (sym < 256u) {
    pb_drop(r, L);
    v = sym;
    return 0;
  }
  if (sym == 256u) {
    pb_drop(r, L);
    return 2;
  }
  if (sym > 285u) {
    pb_drop(r, L);
    return 3;
  }
  uint32_t lbase, lext;
  length_base(sym, lbase, lext);
  v = lbase + (((uint32_t)(r.b.bb >> L)) & ((1u << lext) - 1u));
  pb_drop(r, L + lext);
  br_refill(r.b);
  e = s.d[(uint32_t)r.b.bb & ((1u << PI_D_ROOT) - 1)];
  L = e & 15u;
  uint32_t dsym = e >> 4;
  if (L == 0) dsym = pi_long(s.lim_d, s.off_d, s.sd, PI_D_ROOT, r.b.bb, L);
  if (dsym > 29u) {
    pb_drop(r, L);
    return 3;
  }
  uint32_t dbase, dext;
  dist_base(dsym, dbase, dext);
  w = dbase + (((uint32_t)(r.b.bb >> L)) & ((1u << dext) - 1u));
  pb_drop(r, L + dext);
  return 1;
}

// ---- canonical tables from s.lens[base .. base+n) into the LL (which=0) or D (which=1)
// lookup.  Returns false (uniform) unless the code is complete (the only kind zlib and
// libdeflate emit; anything else takes the exact path).
__device__ bool pi_build(PiShared& s, uint32_t base, uint32_t n, uint32_t which) {
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint32_t root = which ? PI_D_ROOT : PI_LL_ROOT;
  uint16_t* lut = which ? s.d : s.ll;
  uint16_t* sorted = which ? s.sd : s.sll;
  uint32_t* lim = which ? s.lim_d : s.lim_ll;
  int32_t* off = which ? s.off_d : s.off_ll;
  // zero the table (uint4 stores)
  for (uint32_t i = tid; i < (1u << root) / 8u; i += PI_NL) ((uint4*)lut)[i] = make_uint4(0, 0, 0, 0);
  // wave 0: ranks in symbol order -> codes, counts, sorted symbols
  if (tid < 64) {
    uint32_t run = 0;  // lane L holds the running count of length L
    for (uint32_t c0 = 0; c0 < n; c0 += 64) {
      const uint32_t sidx = c0 + lane;
      const uint32_t len = sidx < n ? s.lens[base + sidx] : 0u;
      uint32_t rank = 0, mycnt = 0;
      const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
      for (uint32_t L = 1; L < 16; ++L) {
        const uint64_t m = __ballot(len == L);
        if (len == L) rank = (uint32_t)__popcll(m & lt);
        if (lane == L) mycnt = (uint32_t)__popcll(m);
      }
      const uint32_t before = __shfl(run, (int)len);
      if (sidx < n) s.codes[sidx] = (uint16_t)(before + rank);  // rank among length-len symbols
      run += mycnt;
    }
    // lane L: count of length L
    const uint32_t cntL = (lane >= 1 && lane < 16) ? run : 0u;
    if (lane < 16) s.cnt[which][lane] = cntL;
  }
  __syncthreads();
  // uniform: completeness, first codes, offsets
  uint32_t first[16];
  int32_t left = 1;
  uint32_t code = 0, nshort = 0;
  bool ok = true;
#pragma unroll
  for (uint32_t L = 1; L < 16; ++L) {
    const uint32_t c = s.cnt[which][L];
    left = 2 * left - (int32_t)c;
    ok &= left >= 0;
    first[L] = code;
    if (tid == 0) {
      lim[L] = (code + c) << (15u - L);
      off[L] = (int32_t)nshort - (int32_t)code;
    }
    nshort += c;
    code = (code + c) << 1;
  }
  if (!ok || left != 0) return false;  // over-subscribed or incomplete (uniform)
  // symbols: sorted table + lookup entries
  for (uint32_t sidx = tid; sidx < n; sidx += PI_NL) {
    const uint32_t len = s.lens[base + sidx];
    if (!len) continue;
    const uint32_t rk = s.codes[sidx];
    uint32_t cl = 0;
#pragma unroll
    for (uint32_t L = 1; L < 16; ++L) cl = (len == L) ? first[L] : cl;
    const uint32_t cd = cl + rk;
    uint32_t nsh = 0;
#pragma unroll
    for (uint32_t L = 1; L < 16; ++L) nsh += (L < len) ? s.cnt[which][L] : 0u;
    sorted[nsh + rk] = (uint16_t)sidx;
    if (len <= root) {
      const uint32_t rev = __builtin_bitreverse32(cd) >> (32u - len);
      const uint16_t ent = (uint16_t)(len | sidx << 4);
      for (uint32_t j = 0; j < (1u << (root - len)); ++j) lut[rev | j << len] = ent;
    }
  }
  return true;
}

// Sink of pass 2: literals / descriptors into ubuf (16-byte write-combining, partial chunks
// at the lane's range edges bytewise), match starts into the LDS bitmap.
struct PiSink {
  uint8_t* ubuf;
  uint64_t u0;        // block start in ubuf
  uint64_t rs, re;    // this lane's absolute output range
  uint64_t cur, lo, hi;
  uint32_t* bm;
  uint32_t bw, bword;
  __device__ __forceinline__ void flush() {
    if (cur == ~0ULL) return;
    if (cur >= rs && cur + 16 <= re) {
      uint4 v;
      v.x = (uint32_t)lo; v.y = (uint32_t)(lo >> 32); v.z = (uint32_t)hi; v.w = (uint32_t)(hi >> 32);
      *(uint4*)(ubuf + cur) = v;
    } else {
      for (uint32_t k = 0; k < 16; ++k) {
        const uint64_t a = cur + k;
        if (a >= rs && a < re) ubuf[a] = (uint8_t)((k < 8 ? lo >> (8 * k) : hi >> (8 * (k - 8))) & 0xff);
      }
    }
  }
  __device__ __forceinline__ void put(uint32_t op, uint32_t b) {
    const uint64_t a = u0 + op;
    const uint64_t c = a & ~15ULL;
    if (c != cur) {
      flush();
      cur = c;
      lo = 0;
      hi = 0;
    }
    const uint32_t k = (uint32_t)(a & 15);
    if (k < 8) lo |= (uint64_t)(b & 0xff) << (8 * k);
    else hi |= (uint64_t)(b & 0xff) << (8 * (k - 8));
  }
  __device__ __forceinline__ void mark(uint32_t op) {
    const uint32_t wi = op >> 5;
    if (wi != bw) {
      if (bword) atomicOr(&bm[bw], bword);
      bw = wi;
      bword = 0;
    }
    bword |= 1u << (op & 31);
  }
  __device__ __forceinline__ void finish() {
    flush();
    if (bword) atomicOr(&bm[bw], bword);
  }
};

// Per-launch counters (device, u64): [0] retried blocks (set by the kernel), [1] rounds,
// [2] DEFLATE headers, [3] commits ended by a sync failure, [4] by an EOB-list overflow,
// [5..9] shader cycles in header / pass 1 / sync / plan / pass 2, [10] blocks,
// [11] active lanes summed over rounds, [12] committing lane summed over rounds.
constexpr uint32_t PI_NSTAT = 13;
struct PiStat {
  uint64_t v[PI_NSTAT];
};
#define PI_CLK() __builtin_amdgcn_s_memtime()

// Whole-block decode.  Returns INF_OK (tokens written, bitmap in s.bm) or INF_RETRY.
__device__ int32_t inflate_par_block(PiShared& s, const uint8_t* __restrict__ cdata, uint32_t nbytes,
                                     uint32_t isize, uint8_t* __restrict__ ubuf, uint64_t u0,
                                     PiStat& ps) {
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint32_t wave = tid >> 6;
  const uint32_t T = nbytes * 8u;
  for (uint32_t i = tid; i < BITMAP_WORDS; i += PI_NL) s.bm[i] = 0;
  uint32_t pos = 0, op = 0;
  bool in_block = false, final_blk = false;
  uint32_t rounds = 0;
  __syncthreads();
  for (;;) {
    if (!in_block) {
      if (final_blk) break;
      const uint64_t c0 = PI_CLK();
      ps.v[2] += 1;
      // ---- block header (every lane decodes the same bits: uniform values)
      if (pos + 3 > T) return INF_RETRY;
      PBits h;
      pb_init(h, cdata, pos);
      br_refill(h.b);
      final_blk = (h.b.bb & 1u) != 0;
      const uint32_t type = (uint32_t)(h.b.bb >> 1) & 3u;
      pb_drop(h, 3);
      if (type == 0u) {
        const uint32_t bytepos = (h.pos + 7u) >> 3;
        if (bytepos * 8u + 32u > T) return INF_RETRY;
        const uint8_t* p = cdata + bytepos;
        const uint32_t len = (uint32_t)p[0] | (uint32_t)p[1] << 8;
        const uint32_t nlen = (uint32_t)p[2] | (uint32_t)p[3] << 8;
        if (len != (nlen ^ 0xffffu)) return INF_RETRY;
        if ((bytepos + 4u + len) * 8u > T || op + len > isize) return INF_RETRY;
        for (uint32_t k = tid; k < len; k += PI_NL) ubuf[u0 + op + k] = p[4 + k];
        op += len;
        pos = (bytepos + 4u + len) * 8u;
        __syncthreads();
        continue;
      }
      if (type == 3u) return INF_RETRY;
      uint32_t nlen = 288, ndist = 32;
      if (type == 1u) {
        for (uint32_t k = tid; k < 320; k += PI_NL)
          s.lens[19 + k] = (uint8_t)(k < 144 ? 8 : k < 256 ? 9 : k < 280 ? 7 : 8 - (k >= 288 ? 3 : 0));
      } else {
        br_refill(h.b);
        nlen = ((uint32_t)h.b.bb & 31u) + 257u;
        ndist = ((uint32_t)(h.b.bb >> 5) & 31u) + 1u;
        const uint32_t ncode = ((uint32_t)(h.b.bb >> 10) & 15u) + 4u;
        pb_drop(h, 14);
        if (nlen > 286u || ndist > 30u) return INF_RETRY;
        // code-length code lengths
        const uint64_t ord_lo = 0x022caa324e804a30ULL, ord_hi = 0x00000003c2e1346cULL;
        if (tid < 19) s.lens[tid] = 0;
        for (uint32_t k = tid; k < 128; k += PI_NL) s.cl[k] = 0;
        __syncthreads();
        for (uint32_t i = 0; i < ncode; ++i) {
          br_refill(h.b);
          const uint32_t o = (uint32_t)((i < 12u ? ord_lo >> (5u * i) : ord_hi >> (5u * (i - 12u))) & 31u);
          if (tid == 0) s.lens[o] = (uint8_t)(h.b.bb & 7u);
          pb_drop(h, 3);
        }
        __syncthreads();
        // CL table: complete code, 7-bit root (lane-per-symbol fill)
        {
          uint32_t cnt[8];
#pragma unroll
          for (int L = 0; L < 8; ++L) cnt[L] = 0;
          for (uint32_t k = 0; k < 19; ++k) {
            const uint32_t l = s.lens[k];
#pragma unroll
            for (int L = 1; L < 8; ++L) cnt[L] += (l == (uint32_t)L) ? 1u : 0u;
          }
          int32_t left = 1;
          bool ok = true;
          uint32_t first[8], code = 0;
#pragma unroll
          for (int L = 1; L < 8; ++L) {
            left = 2 * left - (int32_t)cnt[L];
            ok &= left >= 0;
            first[L] = code;
            code = (code + cnt[L]) << 1;
          }
          if (!ok || left != 0) return INF_RETRY;
          if (tid < 19) {
            const uint32_t l = s.lens[tid];
            if (l) {
              uint32_t rk = 0;
              for (uint32_t k = 0; k < tid; ++k) rk += (s.lens[k] == l) ? 1u : 0u;
              uint32_t f = 0;
#pragma unroll
              for (int L = 1; L < 8; ++L) f = (l == (uint32_t)L) ? first[L] : f;
              const uint32_t rev = __builtin_bitreverse32(f + rk) >> (32u - l);
              for (uint32_t j = 0; j < (1u << (7u - l)); ++j) s.cl[rev | j << l] = (uint16_t)(l | tid << 4);
            }
          }
        }
        __syncthreads();
        // HLIT + HDIST code lengths (sequential, uniform)
        const uint32_t total = nlen + ndist;
        uint32_t have = 0, prev = 0;
        while (have < total) {
          br_refill(h.b);
          if (h.pos >= T) return INF_RETRY;
          const uint32_t e = s.cl[(uint32_t)h.b.bb & 127u];
          const uint32_t L = e & 15u, sym = e >> 4;
          pb_drop(h, L);
          if (sym < 16u) {
            if (tid == 0) s.lens[19 + have] = (uint8_t)sym;
            prev = sym;
            ++have;
            continue;
          }
          uint32_t rep, val = 0;
          if (sym == 16u) {
            if (have == 0) return INF_RETRY;
            val = prev;
            rep = 3u + ((uint32_t)h.b.bb & 3u);
            pb_drop(h, 2);
          } else if (sym == 17u) {
            rep = 3u + ((uint32_t)h.b.bb & 7u);
            pb_drop(h, 3);
          } else {
            rep = 11u + ((uint32_t)h.b.bb & 127u);
            pb_drop(h, 7);
          }
          if (have + rep > total) return INF_RETRY;
          if (tid == 0)
            for (uint32_t k = 0; k < rep; ++k) s.lens[19 + have + k] = (uint8_t)val;
          have += rep;
          prev = val;
        }
        if (h.pos > T) return INF_RETRY;
        __syncthreads();
        if (s.lens[19 + 256] == 0) return INF_RETRY;
      }
      __syncthreads();
      if (!pi_build(s, 19, nlen, 0)) return INF_RETRY;
      __syncthreads();
      if (!pi_build(s, 19 + nlen, ndist, 1)) return INF_RETRY;
      __syncthreads();
      pos = h.pos;
      in_block = true;
      ps.v[5] += PI_CLK() - c0;
    }
    if (++rounds > PI_MAX_ROUNDS || pos >= T) return INF_RETRY;
    ps.v[1] += 1;
    const uint64_t c1 = PI_CLK();

    // ---- pass 1: segments of [pos, T)
    const uint32_t R = T - pos;
    uint32_t seg = (R + PI_NL - 1) / PI_NL;
    if (seg < PI_MIN_SEG) seg = PI_MIN_SEG;
    const uint32_t nact = (R + seg - 1) / seg;  // active lanes
    const uint32_t s0 = pos + tid * seg;
    const uint32_t lim = (tid + 1 < nact) ? s0 + seg : T;
    PBits r;
    uint32_t bytes = 0;
    if (tid < nact) {
      pb_init(r, cdata, s0);
      uint32_t nb = 0, ne = 0;
      while (r.pos < lim) {
        const uint32_t st = r.pos;
        uint32_t v, w;
        const uint32_t k = pi_token(s, r, v, w);
        if (nb < PI_M) s.bdel[tid * PI_M + nb++] = (uint8_t)(r.pos - st);
        if (k == 0) bytes += 1;
        else if (k == 1) bytes += v;
        else if (k == 2) {
          if (ne < PI_E) {
            s.eob_s[tid * PI_E + ne] = st;
            s.eob_e[tid * PI_E + ne] = r.pos;
            s.eob_c[tid * PI_E + ne] = bytes;
          }
          ++ne;
        }
      }
      s.nbnd[tid] = (uint8_t)nb;
      s.neob[tid] = (uint8_t)(ne > 255 ? 255 : ne);
      s.tot[tid] = bytes;
    }
    __syncthreads();
    const uint64_t c2 = PI_CLK();
    ps.v[6] += c2 - c1;
    ps.v[11] += nact;
    // ---- sync with the next lane
    if (tid < nact) {
      uint32_t sp = PI_NONE, sc = 0;
      if (tid + 1 < nact) {
        // lane i+1's token starts: t_0 = s1, t_{j+1} = t_j + bdel[j], j < nb1
        const uint32_t nb1 = s.nbnd[tid + 1];
        const uint8_t* del = s.bdel + (tid + 1) * PI_M;
        uint32_t j = 0, p1 = s0 + seg, ne = s.neob[tid];
        for (;;) {
          const uint32_t q = r.pos;
          while (j < nb1 && p1 < q) p1 += del[j++];
          if (p1 == q) {
            sp = q;
            sc = j;
            break;
          }
          if (p1 < q || q >= T) break;  // lane i+1's recorded starts exhausted
          uint32_t v, w;
          const uint32_t k = pi_token(s, r, v, w);
          if (k == 0) bytes += 1;
          else if (k == 1) bytes += v;
          else if (k == 2) {
            if (ne < PI_E) {
              s.eob_s[tid * PI_E + ne] = q;
              s.eob_e[tid * PI_E + ne] = r.pos;
              s.eob_c[tid * PI_E + ne] = bytes;
            }
            ++ne;
            break;  // the stream changes meaning after an end-of-block code
          }
        }
        s.neob[tid] = (uint8_t)(ne > 255 ? 255 : ne);
      }
      s.syn_pos[tid] = sp;
      s.syn_idx[tid] = sc;
      s.syn_bytes[tid] = bytes;
      s.syn_stop[tid] = r.pos;
    }
    if (tid == 0) {
      s.u[0] = PI_NONE;  // first stopping lane
      s.u[4] = 0;        // pass-2 failure flag
    }
    __syncthreads();
    const uint64_t c3 = PI_CLK();
    ps.v[7] += c3 - c2;
    // ---- plan: per-lane true start, stop condition
    uint32_t P = 0, before = 0, kind = 0, nbytes_l = 0, endbit = 0, nextpos = 0;
    // kind: 0 continue (synced, no EOB), 1 ends with EOB, 2 stops (sync failure), 3 unknown
    if (tid < nact) {
      P = tid == 0 ? pos : s.syn_pos[tid - 1];
      const bool live = (tid == 0) || (P != PI_NONE);
      if (live && tid) {
        // bytes of this lane's decode before P: re-decode its first syn_idx tokens
        PBits q;
        pb_init(q, cdata, s0);
        const uint32_t nt = s.syn_idx[tid - 1];
        for (uint32_t t = 0; t < nt; ++t) {
          uint32_t v, w;
          const uint32_t k = pi_token(s, q, v, w);
          before += (k == 0) ? 1u : (k == 1) ? v : 0u;
        }
        if (q.pos != P) atomicOr(&s.u[4], 1u);  // cannot happen: P is one of its starts
      }
      if (live) {
        const uint32_t ne = s.neob[tid];
        const uint32_t nrec = ne < PI_E ? ne : PI_E;
        bool found = false;
        for (uint32_t k = 0; k < nrec && !found; ++k) {
          if (s.eob_s[tid * PI_E + k] >= P) {
            found = true;
            endbit = s.eob_s[tid * PI_E + k];
            nextpos = s.eob_e[tid * PI_E + k];
            nbytes_l = s.eob_c[tid * PI_E + k] - before;
          }
        }
        if (found) kind = 1;
        else if (ne > PI_E) kind = 3;
        else if (s.syn_pos[tid] == PI_NONE) {
          kind = 2;
          endbit = s.syn_stop[tid];
          nextpos = endbit;
          nbytes_l = s.syn_bytes[tid] - before;
        } else {
          kind = 0;
          endbit = s.syn_pos[tid];
          nbytes_l = s.syn_bytes[tid] - before;
        }
        if (kind) atomicMin(&s.u[0], tid);
      }
    }
    __syncthreads();
    const uint32_t e = s.u[0];
    if (e == PI_NONE) return INF_RETRY;  // cannot happen: the last active lane never syncs
    if (tid == e) {
      s.u[1] = kind;
      s.u[2] = nextpos;
      s.u[3] = P;
    }
    // commit lanes [0, ncommit)
    __syncthreads();
    const uint32_t ekind = s.u[1];
    const uint32_t ncommit = (ekind == 3) ? e : e + 1;
    const bool mine = tid < ncommit;
    const uint32_t myb = mine ? nbytes_l : 0u;
    // block-wide exclusive scan of myb
    uint32_t incl = myb;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o);
      if ((int)lane >= o) incl += t;
    }
    if (lane == 63) s.wsum[wave] = incl;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
    for (uint32_t w = 0; w < PI_WAVES; ++w) {
      const uint32_t x = s.wsum[w];
      wbase += (w < wave) ? x : 0u;
      total += x;
    }
    const uint32_t obase = op + wbase + incl - myb;
    if (op + total > isize) return INF_RETRY;
    const uint64_t c4 = PI_CLK();
    ps.v[8] += c4 - c3;
    ps.v[12] += e;
    ps.v[3] += (ekind == 2);
    ps.v[4] += (ekind == 3);
    // ---- pass 2: emit
    bool bad = false;
    if (mine && myb) {
      PBits q;
      pb_init(q, cdata, P);
      PiSink sk;
      sk.ubuf = ubuf;
      sk.u0 = u0;
      sk.rs = u0 + obase;
      sk.re = u0 + obase + myb;
      sk.cur = ~0ULL;
      sk.lo = 0;
      sk.hi = 0;
      sk.bm = s.bm;
      sk.bw = 0;
      sk.bword = 0;
      uint32_t o = obase;
      const uint32_t oend = obase + myb;
      while (q.pos < endbit) {
        uint32_t v, w;
        const uint32_t k = pi_token(s, q, v, w);
        if (k == 0) {
          if (o >= oend) { bad = true; break; }
          sk.put(o, v);
          ++o;
        } else if (k == 1) {
          if (w > o || o + v > oend) { bad = true; break; }
          const uint32_t dd = w - 1;
          sk.put(o, v - 3);
          sk.put(o + 1, dd & 0xff);
          sk.put(o + 2, dd >> 8);
          sk.mark(o);
          o += v;
        } else {
          bad = true;
          break;
        }
      }
      sk.finish();
      if (q.pos != endbit || o != oend) bad = true;
    } else if (mine && P != endbit) {
      bad = true;  // every token but end-of-block yields bytes: a byte-less region is empty
    }
    if (bad) atomicOr(&s.u[4], 1u);
    __syncthreads();
    if (s.u[4]) return INF_RETRY;
    ps.v[9] += PI_CLK() - c4;
    op += total;
    pos = s.u[2];
    if (ekind == 3) pos = s.u[3];
    if (ekind == 1) in_block = false;
    if (pos > T) return INF_RETRY;
    __syncthreads();
  }
  if (op != isize || pos > T) return INF_RETRY;
  return INF_OK;
}

}  // namespace hbam
