// hbam_deflate.hip — BGZF block compression on the device: the
// BlockCompressedOutputStream under BAMRecordWriter (BAMRecordWriter.java:96-111) and
// SAMOutputPreparer (util/SAMOutputPreparer.java:58-95), for the Sort plugin's output.
//
// The uncompressed stream is cut into blocks of `bsize` bytes; every block becomes one
// independent BGZF member (RFC 1952 header with the BC extra field, one raw DEFLATE stream,
// CRC32, ISIZE).  Parity is defined on the inflated bytes: any valid
// DEFLATE stream is accepted by htsjdk's reader, so the compressor is free to be GPU-shaped.
//
//   k_lz77_tokens (one 256-thread workgroup per block): the block is staged in LDS; for every
//     256-position chunk each thread probes (up to 16 bytes) the most recent earlier position
//     with the same 4-byte hash (from earlier chunks) and the four previous positions (byte /
//     short-period runs), extending a match the probe capped to its full length; the
//     greedy parse of the chunk is then found by pointer jumping over the successor of each
//     position (2^k-th successors, then the path from the entry marked level by level), and
//     every thread writes its position's token at its rank.  Tokens go to a per-block global
//     buffer.
//   k_deflate_encode (one 256-thread workgroup per block): symbol frequencies from the
//     tokens, length-limited Huffman codes (lit/len ≤ 15, distance ≤ 15, code-length code ≤ 7), the dynamic-block
//     header, then every token's bit offset by a block-wide scan and its bits OR-ed into an
//     LDS output image; a block that does not shrink is written as a stored block.  The
//     BGZF member goes to a 64 KiB slot; a scan + copy packs the slots.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbam_internal.h"

namespace hbam {

constexpr uint32_t DF_WG = 256;
constexpr uint32_t DF_MAXB = 65280;           // largest block accepted (bgzip's 0xff00)
constexpr uint32_t DF_HBITS = 11;             // 2048-entry hash heads
constexpr uint32_t DF_SLOT = 65536;           // BGZF member slot (BSIZE <= 65536)
constexpr uint32_t DF_NSYM = 286 + 30;        // lit/len + distance frequencies per block
constexpr uint32_t DF_WINDOW = 32768;
constexpr uint32_t DF_PROBE = 16;             // match bytes verified per position in parallel

__device__ __forceinline__ uint32_t df_hash(uint32_t w) { return (w * 2654435761u) >> (32 - DF_HBITS); }

__device__ __forceinline__ uint32_t df_rd32(const uint8_t* s, uint32_t p) {
  return (uint32_t)s[p] | (uint32_t)s[p + 1] << 8 | (uint32_t)s[p + 2] << 16 | (uint32_t)s[p + 3] << 24;
}
// unaligned dword from LDS (the device runs in unaligned access mode, as k_resolve relies on)
__device__ __forceinline__ uint32_t df_lds32(const uint8_t* s, uint32_t p) { return *(const uint32_t*)(s + p); }

// length of the common prefix of s[a..] and s[p..], at most lim
__device__ __forceinline__ uint32_t df_match(const uint8_t* s, uint32_t a, uint32_t p, uint32_t lim) {
  uint32_t l = 0;
  while (l + 4 <= lim) {
    const uint32_t x = df_lds32(s, a + l) ^ df_lds32(s, p + l);
    if (x) return l + (__builtin_ctz(x) >> 3);
    l += 4;
  }
  while (l < lim && s[a + l] == s[p + l]) ++l;
  return l;
}

// RFC 1951 length code of a match length 3..258: symbol, extra bits, extra value
__device__ __forceinline__ void df_len_code(uint32_t len, uint32_t& sym, uint32_t& eb, uint32_t& ev) {
  if (len == 258) {
    sym = 285; eb = 0; ev = 0;
    return;
  }
  const uint32_t x = len - 3;
  if (x < 8) {
    sym = 257 + x; eb = 0; ev = 0;
    return;
  }
  eb = 31 - __builtin_clz(x) - 2;  // x in [8, 255]: 1..5 extra bits
  const uint32_t base = (4u + ((x >> eb) & 3u)) << eb;
  sym = 257 + 4 * eb + 4 + ((x >> eb) & 3u);
  ev = x - base;
}
// distance code of 1..32768
__device__ __forceinline__ void df_dist_code(uint32_t d, uint32_t& sym, uint32_t& eb, uint32_t& ev) {
  const uint32_t x = d - 1;
  if (x < 4) {
    sym = x; eb = 0; ev = 0;
    return;
  }
  eb = 31 - __builtin_clz(x) - 1;  // x in [4, 32767]: 1..13 extra bits
  const uint32_t hb = (x >> eb) & 1u;
  sym = 2 * eb + 2 + hb;
  ev = x - ((2u + hb) << eb);
}

#ifdef HBAM_PROF
__device__ unsigned long long* g_dfprof = nullptr;  // 8 u64 per block (tools/prof_deflate.py)
#define DF_T() __builtin_amdgcn_s_memtime()
#endif
// token: literal = byte; match = 1<<31 | len<<16 | dist (dist <= 32768, len <= 258)
__global__ __launch_bounds__(DF_WG) void k_lz77_tokens(const uint8_t* __restrict__ src, uint64_t n,
                                                       uint32_t bsize, uint32_t nblk,
                                                       uint32_t* __restrict__ tok,
                                                       uint32_t* __restrict__ ntok) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[DF_MAXB + 288];
  __shared__ uint32_t s_head[1u << DF_HBITS];
  __shared__ uint32_t s_ml[DF_WG];
  __shared__ uint16_t s_jmp[8][DF_WG];  // 2^k-th successor in the greedy parse
  __shared__ uint32_t s_vis[8];         // token starts of the chunk
  const uint32_t b = blockIdx.x, t = threadIdx.x;
  if (b >= nblk) return;
  const uint64_t start = (uint64_t)b * bsize;
  const uint32_t len = (uint32_t)((n - start) < bsize ? (n - start) : bsize);
  const uint8_t* sb = src + start;
  if (((uintptr_t)sb & 15u) == 0) {  // 16-byte loads (the caller's buffer is usually aligned)
    for (uint32_t i = t; i < (DF_MAXB + 288) / 16; i += DF_WG) {
      const uint32_t p = 16 * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (p + 16 <= len) {
        v = *(const uint4*)(sb + p);
      } else if (p < len) {
        uint32_t w[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; p + k < len; ++k) w[k >> 2] |= (uint32_t)sb[p + k] << (8 * (k & 3u));
        v = make_uint4(w[0], w[1], w[2], w[3]);
      }
      ((uint4*)s_in)[i] = v;
    }
  } else {
    for (uint32_t i = t; i < (DF_MAXB + 288) / 4; i += DF_WG) {
      const uint32_t p = 4 * i;
      uint32_t w = 0;
      for (uint32_t k = 0; k < 4; ++k)
        if (p + k < len) w |= (uint32_t)sb[p + k] << (8 * k);
      ((uint32_t*)s_in)[i] = w;
    }
  }
  for (uint32_t i = t; i < (1u << DF_HBITS); i += DF_WG) s_head[i] = 0;
  __syncthreads();
  uint32_t* out = tok + (uint64_t)b * bsize;
  uint32_t nxt = 0, nt = 0;  // parse position / tokens emitted (wave 0, uniform)
#ifdef HBAM_PROF
  uint64_t pt0 = DF_T(), p_match = 0, p_walk = 0, p_sync = 0, n_iter = 0, tq;
#endif
  for (uint32_t c0 = 0; c0 < len; c0 += DF_WG) {
#ifdef HBAM_PROF
    const uint64_t tm0 = DF_T();
#endif
    const uint32_t p = c0 + t;
    uint32_t best = 0;
    uint32_t h = 0;
    const bool has4 = p + 4 <= len;
    if (has4) {
      // lengths are found up to DF_PROBE bytes for every position; the parse extends the
      // matches it takes (only those) to their full length
      const uint32_t lim = (len - p) < DF_PROBE ? (len - p) : DF_PROBE;
      h = df_hash(df_lds32(s_in, p));
      uint32_t bl = 0, bd = 0;
      // short periods first: runs of one byte and of short repeats are the commonest match
#pragma unroll
      for (uint32_t d = 1; d <= 4; ++d) {
        if (p >= d) {
          const uint32_t m = df_match(s_in, p - d, p, lim);
          if (m > bl) {
            bl = m;
            bd = d;
          }
        }
      }
      const uint32_t hc = s_head[h];
      if (hc) {
        const uint32_t a = hc - 1;
        if (p - a <= DF_WINDOW && p - a > 4) {
          const uint32_t m = df_match(s_in, a, p, lim);
          if (m > bl) {
            bl = m;
            bd = p - a;
          }
        }
      }
      if (bl >= 4 || (bl == 3 && bd <= 64)) {
        if (bl == DF_PROBE) {  // the probe capped it: this position's full length (<= 258)
          const uint32_t full = (len - p) < 258u ? (len - p) : 258u;
          bl += df_match(s_in, p - bd + DF_PROBE, p + DF_PROBE, full - DF_PROBE);
        }
        best = 0x80000000u | bl << 16 | bd;
      }
    }
    s_ml[t] = best;
#ifdef HBAM_PROF
    tq = DF_T();
    p_match += tq - tm0;
#endif
    // successor of each position in the greedy parse (256 = past the chunk)
    const uint32_t cend = (c0 + DF_WG < len) ? c0 + DF_WG : len;
    {
      const uint32_t step = best ? (best >> 16) & 0x1ffu : 1u;
      const uint32_t nx = t + step;
      s_jmp[0][t] = (uint16_t)((p < cend && c0 + nx < cend) ? nx : DF_WG);
    }
    if (t < 8) s_vis[t] = 0;
    __syncthreads();
#ifdef HBAM_PROF
    {
      const uint64_t t2 = DF_T();
      p_sync += t2 - tq;
      tq = t2;
    }
#endif
    if (has4) atomicMax(&s_head[h], p + 1);  // most recent position of the hash, for later chunks
    // Greedy parse of the chunk from nxt by pointer jumping: jmp[k][i] = the 2^k-th successor
    // of i; then the token starts = steps 0.. of the path from nxt, found from the most
    // significant jump down (after level k the set holds every step that is a multiple of
    // 2^k), then every thread emits its position's token at its rank among the starts.
#pragma unroll 1
    for (uint32_t k = 1; k < 8; ++k) {
      const uint32_t j = s_jmp[k - 1][t];
      s_jmp[k][t] = j < DF_WG ? s_jmp[k - 1][j] : (uint16_t)DF_WG;
      __syncthreads();
    }
    const uint32_t e = nxt - c0;  // nxt is uniform: every thread tracks it
    if (nxt < cend) {
      if (t == 0) s_vis[e >> 5] = 1u << (e & 31u);
      __syncthreads();
#pragma unroll 1
      for (int k = 7; k >= 0; --k) {
        if ((s_vis[t >> 5] >> (t & 31u)) & 1u) {
          const uint32_t j = s_jmp[k][t];
          if (j < DF_WG) atomicOr(&s_vis[j >> 5], 1u << (j & 31u));
        }
        __syncthreads();
      }
      // rank of each start: whole words before + bits below in its word
      const uint32_t w = t >> 5, bit = t & 31u;
      uint32_t before = 0, total = 0;
#pragma unroll
      for (uint32_t q = 0; q < 8; ++q) {
        const uint32_t c = (uint32_t)__popc(s_vis[q]);
        before += q < w ? c : 0u;
        total += c;
      }
      const uint32_t vw = s_vis[w];
      if ((vw >> bit) & 1u) {
        before += (uint32_t)__popc(vw & ((1u << bit) - 1u));
        out[nt + before] = best ? best : (uint32_t)s_in[p];
      }
      // the last start's successor is where the next chunk's parse begins
      uint32_t last = 0;
#pragma unroll
      for (int q = 7; q >= 0; --q) {
        if (s_vis[q]) {
          last = 32u * (uint32_t)q + 31u - (uint32_t)__clz(s_vis[q]);
          break;
        }
      }
      const uint32_t lm = s_ml[last];
      nt += total;
      nxt = c0 + last + (lm ? (lm >> 16) & 0x1ffu : 1u);
#ifdef HBAM_PROF
      n_iter += total;
#endif
    }
#ifdef HBAM_PROF
    {
      const uint64_t t2 = DF_T();
      p_walk += t2 - tq;
      tq = t2;
    }
#endif
    __syncthreads();
  }
  if (t == 0) ntok[b] = nt;
#ifdef HBAM_PROF
  if (g_dfprof && t == 0) {
    unsigned long long* g = g_dfprof + 8 * (uint64_t)b;
    g[0] = DF_T() - pt0;
    g[1] = p_walk;
    g[2] = p_sync;
    g[3] = n_iter;
    g[4] = nt;
    g[5] = p_match;
  }
#endif
}

// ---- Huffman code lengths (one thread): Huffman tree by two queues over the symbols sorted
// by frequency, then lengths limited to maxl.  sorted[] / wt[] / par[] are LDS scratch.
__device__ void df_lengths(const uint32_t* f, uint32_t n, uint32_t maxl, uint8_t* len,
                           uint16_t* sorted, uint32_t* wt, uint16_t* par, uint32_t m) {
  // m = number of used symbols (listed in sorted[0..m) by ascending frequency)
  for (uint32_t i = 0; i < n; ++i) len[i] = 0;
  if (m == 0) return;
  if (m == 1) {
    len[sorted[0]] = 1;
    return;
  }
  // nodes: 0..m-1 leaves (in sorted order), m..2m-2 internal; two-queue merge
  for (uint32_t i = 0; i < m; ++i) wt[i] = f[sorted[i]];
  uint32_t ql = 0, qi = m, ni = m;
  for (uint32_t k = 0; k < m - 1; ++k) {
    uint32_t pick[2];
    for (int j = 0; j < 2; ++j) {
      if (ql < m && (qi >= ni || wt[ql] <= wt[qi])) pick[j] = ql++;
      else pick[j] = qi++;
    }
    wt[ni] = wt[pick[0]] + wt[pick[1]];
    par[pick[0]] = (uint16_t)ni;
    par[pick[1]] = (uint16_t)ni;
    ++ni;
  }
  // depths: root = ni - 1
  uint32_t* dep = wt;  // reuse: depth of node i (computed top-down: parents have larger ids)
  dep[ni - 1] = 0;
  for (int i = (int)ni - 2; i >= 0; --i) dep[i] = dep[par[i]] + 1;
  // bit-length counts, limited to maxl with zlib's repair step (trees.c gen_bitlen): leaves
  // deeper than maxl are clamped to maxl, which over-subscribes the code; each repair step
  // moves a leaf from the deepest level L < maxl down to L+1 and a leaf from maxl up beside
  // it, lowering the Kraft sum (in units of 2^-maxl) by exactly one.  The step count is the
  // Kraft excess itself, so the result is complete (inflate rejects incomplete lit/len and
  // code-length sets).  (r02 counted only the clamped leaves, which under-repairs any
  // subtree of 4+ leaves below depth maxl: ADVICE r02.)
  uint32_t cnt[16];
  for (int L = 0; L < 16; ++L) cnt[L] = 0;
  for (uint32_t i = 0; i < m; ++i) {
    const uint32_t d = dep[i];
    ++cnt[d > maxl ? maxl : d];
  }
  uint32_t kraft = 0;
  for (uint32_t L = 1; L <= maxl; ++L) kraft += cnt[L] << (maxl - L);
  for (uint32_t excess = kraft - (1u << maxl); excess > 0u && cnt[maxl] > 0u; --excess) {
    uint32_t L = maxl - 1;
    while (L > 0 && cnt[L] == 0) --L;
    if (L == 0) break;  // cannot happen for m <= 2^maxl leaves (guard)
    --cnt[L];
    cnt[L + 1] += 2;
    --cnt[maxl];
  }
  // lengths by frequency: the least frequent symbols (front of sorted[]) get the longest codes
  uint32_t k = 0;
  for (uint32_t L = maxl; L >= 1; --L)
    for (uint32_t c = 0; c < cnt[L]; ++c) len[sorted[k++]] = (uint8_t)L;
}

// canonical codes, bit-reversed for the LSB-first bit stream
__device__ void df_codes(const uint8_t* len, uint32_t n, uint16_t* code) {
  uint32_t cnt[16], next[16];
  for (int L = 0; L < 16; ++L) cnt[L] = 0;
  for (uint32_t i = 0; i < n; ++i) ++cnt[len[i]];
  cnt[0] = 0;
  uint32_t c = 0;
  for (int L = 1; L < 16; ++L) {
    c = (c + cnt[L - 1]) << 1;
    next[L] = c;
  }
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t L = len[i];
    if (!L) {
      code[i] = 0;
      continue;
    }
    const uint32_t v = next[L]++;
    code[i] = (uint16_t)(__builtin_bitreverse32(v) >> (32 - L));
  }
}

// sort used symbols by (frequency, symbol) ascending into sorted[], parallel ranks
__device__ uint32_t df_sort_used(const uint32_t* f, uint32_t n, uint16_t* sorted, uint32_t t) {
  __shared__ uint32_t s_m;
  if (t == 0) s_m = 0;
  __syncthreads();
  for (uint32_t i = t; i < n; i += DF_WG) {
    if (!f[i]) continue;
    uint32_t r = 0;
    for (uint32_t j = 0; j < n; ++j)
      r += (f[j] && (f[j] < f[i] || (f[j] == f[i] && j < i))) ? 1u : 0u;
    sorted[r] = (uint16_t)i;
    atomicAdd(&s_m, 1u);
  }
  __syncthreads();
  return s_m;
}

struct DfBits {  // serial bit writer into the LDS image (one thread)
  uint32_t* w;
  uint32_t pos;
  __device__ void put(uint32_t v, uint32_t nb) {
    if (!nb) return;
    const uint64_t x = (uint64_t)v << (pos & 31u);
    w[pos >> 5] |= (uint32_t)x;
    if ((pos & 31u) + nb > 32u) w[(pos >> 5) + 1] |= (uint32_t)(x >> 32);
    pos += nb;
  }
};

constexpr uint32_t DF_OUTW = (DF_SLOT + 64) / 4;  // LDS image words

__global__ __launch_bounds__(DF_WG) void k_deflate_encode(const uint8_t* __restrict__ src, uint64_t n,
                                                          uint32_t bsize, uint32_t nblk,
                                                          const uint32_t* __restrict__ tok,
                                                          const uint32_t* __restrict__ ntok,
                                                          const uint32_t* __restrict__ crc,
                                                          uint8_t* __restrict__ slots,
                                                          uint32_t* __restrict__ csize) {
  __shared__ uint32_t s_out[DF_OUTW];
  __shared__ uint32_t s_f[DF_NSYM];
  __shared__ uint8_t s_len[DF_NSYM];
  __shared__ uint16_t s_code[DF_NSYM];
  __shared__ uint16_t s_sorted[320];
  __shared__ uint32_t s_wt[640];
  __shared__ uint16_t s_par[640];
  __shared__ uint32_t s_clf[19];
  __shared__ uint8_t s_cll[19];
  __shared__ uint16_t s_clc[19];
  __shared__ uint16_t s_rle[320];   // RLE'd code lengths: sym | extra << 5
  __shared__ uint32_t s_nrle, s_hlit, s_hdist, s_bits, s_wsum[DF_WG / 64];
  const uint32_t b = blockIdx.x, t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  if (b >= nblk) return;
  const uint64_t start = (uint64_t)b * bsize;
  const uint32_t len = (uint32_t)((n - start) < bsize ? (n - start) : bsize);
  const uint32_t nt = ntok[b];
  const uint32_t* tk = tok + (uint64_t)b * bsize;
  for (uint32_t i = t; i < DF_NSYM; i += DF_WG) s_f[i] = 0;
  for (uint32_t i = t; i < DF_OUTW; i += DF_WG) s_out[i] = 0;
  __syncthreads();
  for (uint32_t i = t; i < nt; i += DF_WG) {  // symbol frequencies of the block's tokens
    const uint32_t x = tk[i];
    if (x & 0x80000000u) {
      uint32_t sy, eb, ev;
      df_len_code((x >> 16) & 0x1ffu, sy, eb, ev);
      atomicAdd(&s_f[sy], 1u);
      df_dist_code(x & 0xffffu, sy, eb, ev);
      atomicAdd(&s_f[286 + sy], 1u);
    } else {
      atomicAdd(&s_f[x], 1u);
    }
  }
  if (t == 0) atomicAdd(&s_f[256], 1u);  // end of block
  __syncthreads();
  if (t == 0) {
    // a complete lit/len code needs two symbols; the end-of-block symbol is always used
    uint32_t used = 0;
    for (uint32_t i = 0; i < 286; ++i) used += s_f[i] ? 1u : 0u;
    if (used < 2) s_f[s_f[0] ? 1 : 0] += 1;
  }
  __syncthreads();
  // lit/len lengths
  uint32_t m = df_sort_used(s_f, 286, s_sorted, t);
  if (t == 0) df_lengths(s_f, 286, 15, s_len, s_sorted, s_wt, s_par, m);
  __syncthreads();
  // distance lengths (an empty set is sent as one unused code of length 1)
  m = df_sort_used(s_f + 286, 30, s_sorted, t);
  if (t == 0) {
    df_lengths(s_f + 286, 30, 15, s_len + 286, s_sorted, s_wt, s_par, m);
    if (m == 0) s_len[286] = 1;
    df_codes(s_len, 286, s_code);
    df_codes(s_len + 286, 30, s_code + 286);
    // HLIT / HDIST and the run-length coded length sequence (RFC 1951 3.2.7)
    uint32_t hlit = 286;
    while (hlit > 257 && !s_len[hlit - 1]) --hlit;
    uint32_t hdist = 30;
    while (hdist > 1 && !s_len[286 + hdist - 1]) --hdist;
    s_hlit = hlit;
    s_hdist = hdist;
    for (int i = 0; i < 19; ++i) s_clf[i] = 0;
    uint32_t nr = 0;
    const uint32_t tot = hlit + hdist;
    uint32_t i = 0;
    while (i < tot) {
      const uint32_t v = i < hlit ? s_len[i] : s_len[286 + i - hlit];
      uint32_t r = 1;
      while (i + r < tot && (i + r < hlit ? s_len[i + r] : s_len[286 + i + r - hlit]) == v) ++r;
      uint32_t left = r;
      if (v == 0) {
        while (left >= 11) {
          const uint32_t k = left < 138 ? left : 138;
          s_rle[nr++] = (uint16_t)(18 | (k - 11) << 5);
          ++s_clf[18];
          left -= k;
        }
        if (left >= 3) {
          s_rle[nr++] = (uint16_t)(17 | (left - 3) << 5);
          ++s_clf[17];
          left = 0;
        }
      } else {
        s_rle[nr++] = (uint16_t)v;
        ++s_clf[v];
        --left;
        while (left >= 3) {
          const uint32_t k = left < 6 ? left : 6;
          s_rle[nr++] = (uint16_t)(16 | (k - 3) << 5);
          ++s_clf[16];
          left -= k;
        }
      }
      while (left) {
        s_rle[nr++] = (uint16_t)v;
        ++s_clf[v];
        --left;
      }
      i += r;
    }
    s_nrle = nr;
    // the code-length code must be complete: at least two symbols
    uint32_t used = 0;
    for (int k = 0; k < 19; ++k) used += s_clf[k] ? 1u : 0u;
    if (used < 2) s_clf[s_clf[0] ? 1 : 0] += 1;
  }
  __syncthreads();
  m = df_sort_used(s_clf, 19, s_sorted, t);
  if (t == 0) {
    df_lengths(s_clf, 19, 7, s_cll, s_sorted, s_wt, s_par, m);
    df_codes(s_cll, 19, s_clc);
    // header
    DfBits bw{s_out, 0};
    bw.put(1, 1);  // BFINAL
    bw.put(2, 2);  // dynamic
    bw.put(s_hlit - 257, 5);
    bw.put(s_hdist - 1, 5);
    const uint8_t ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint32_t hclen = 19;
    while (hclen > 4 && !s_cll[ord[hclen - 1]]) --hclen;
    bw.put(hclen - 4, 4);
    for (uint32_t k = 0; k < hclen; ++k) bw.put(s_cll[ord[k]], 3);
    for (uint32_t k = 0; k < s_nrle; ++k) {
      const uint32_t sy = s_rle[k] & 31u, ex = s_rle[k] >> 5;
      bw.put(s_clc[sy], s_cll[sy]);
      if (sy == 16) bw.put(ex, 2);
      else if (sy == 17) bw.put(ex, 3);
      else if (sy == 18) bw.put(ex, 7);
    }
    s_bits = bw.pos;
  }
  __syncthreads();
  // tokens: each round 256 tokens, bit offsets by a block-wide exclusive scan
  uint32_t base = s_bits;
  bool overflow = false;
  for (uint32_t r0 = 0; r0 < nt; r0 += DF_WG) {
    const uint32_t i = r0 + t;
    uint64_t v = 0;
    uint32_t nb = 0;
    if (i < nt) {
      const uint32_t x = tk[i];
      if (x & 0x80000000u) {
        const uint32_t ml = (x >> 16) & 0x1ffu, d = x & 0xffffu;
        uint32_t sy, eb, ev;
        df_len_code(ml, sy, eb, ev);
        v = s_code[sy];
        nb = s_len[sy];
        v |= (uint64_t)ev << nb;
        nb += eb;
        df_dist_code(d, sy, eb, ev);
        v |= (uint64_t)s_code[286 + sy] << nb;
        nb += s_len[286 + sy];
        v |= (uint64_t)ev << nb;
        nb += eb;
      } else {
        v = s_code[x];
        nb = s_len[x];
      }
    }
    // exclusive scan of nb over the 256 threads
    uint32_t inc = nb;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(inc, off);
      if ((int)lane >= off) inc += y;
    }
    if (lane == 63) s_wsum[wv] = inc;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
    for (uint32_t k = 0; k < DF_WG / 64; ++k) {
      if (k < wv) wbase += s_wsum[k];
      total += s_wsum[k];
    }
    const uint32_t pos = base + wbase + inc - nb;
    if (nb && pos + nb + 16 < 8u * (DF_SLOT - 64)) {
      const uint32_t w = pos >> 5, sh = pos & 31u;
      const uint64_t lo = v << sh;
      const uint32_t hi = sh ? (uint32_t)(v >> (64 - sh)) : 0u;
      atomicOr(&s_out[w], (uint32_t)lo);
      if ((uint32_t)(lo >> 32)) atomicOr(&s_out[w + 1], (uint32_t)(lo >> 32));
      if (hi) atomicOr(&s_out[w + 2], hi);
    }
    base += total;
    if (base + 64 >= 8u * (DF_SLOT - 64)) overflow = true;
    __syncthreads();
  }
  // end of block, then the member
  uint32_t dbytes = 0;
  bool stored = overflow;
  if (!stored) {
    const uint32_t pos = base;
    if (t == 0) {
      DfBits bw{s_out, pos};
      bw.put(s_code[256], s_len[256]);
      s_bits = bw.pos;
    }
    __syncthreads();
    dbytes = (s_bits + 7) >> 3;
    stored = dbytes + 26 > DF_SLOT || dbytes >= len + 5;
  }
  uint8_t* slot = slots + (uint64_t)b * DF_SLOT;
  const uint32_t body = stored ? len + 5 : dbytes;
  const uint32_t total_sz = body + 26;
  if (t == 0) {
    const uint32_t bs1 = total_sz - 1;
    const uint8_t hdr[18] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0,
                             (uint8_t)(bs1 & 0xff), (uint8_t)(bs1 >> 8)};
    for (int k = 0; k < 18; ++k) slot[k] = hdr[k];
    const uint32_t c = crc[b];
    uint8_t* tail = slot + 18 + body;
    for (int k = 0; k < 4; ++k) tail[k] = (uint8_t)(c >> (8 * k));
    for (int k = 0; k < 4; ++k) tail[4 + k] = (uint8_t)(len >> (8 * k));
    if (stored) {  // BFINAL=1 BTYPE=00, byte aligned: LEN, NLEN, the bytes
      slot[18] = 1;
      slot[19] = (uint8_t)(len & 0xff);
      slot[20] = (uint8_t)(len >> 8);
      slot[21] = (uint8_t)(~len & 0xff);
      slot[22] = (uint8_t)((~len >> 8) & 0xff);
    }
    csize[b] = total_sz;
  }
  if (stored) {
    for (uint32_t i = t; i < len; i += DF_WG) slot[23 + i] = src[start + i];
  } else {
    const uint8_t* img = (const uint8_t*)s_out;
    for (uint32_t i = t; i < dbytes; i += DF_WG) slot[18 + i] = img[i];
  }
}

// BGZF members of the blocks -> packed at off[b]
__global__ void k_pack_members(const uint8_t* __restrict__ slots, const uint32_t* __restrict__ csize,
                               const uint64_t* __restrict__ off, uint32_t nblk, uint8_t* __restrict__ dst) {
  const uint32_t b = blockIdx.x;
  if (b >= nblk) return;
  const uint32_t sz = csize[b];
  const uint8_t* s = slots + (uint64_t)b * DF_SLOT;
  uint8_t* d = dst + off[b];
  for (uint32_t i = threadIdx.x; i < sz; i += blockDim.x) d[i] = s[i];
}

// CRC-32 of each uncompressed block (blocks of bsize over src), one thread per block:
// slice-by-4 tables in LDS, 16-byte loads when the block is 16-aligned
__global__ __launch_bounds__(256) void k_crc_blocks(const uint8_t* __restrict__ src, uint64_t n, uint32_t bsize,
                                                    uint32_t nblk, uint32_t* __restrict__ crc_out) {
  __shared__ uint32_t T[4][256];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? 0xedb88320u ^ (c >> 1) : c >> 1;
    T[0][i] = c;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = T[0][i];
    c = T[0][c & 0xff] ^ (c >> 8); T[1][i] = c;
    c = T[0][c & 0xff] ^ (c >> 8); T[2][i] = c;
    c = T[0][c & 0xff] ^ (c >> 8); T[3][i] = c;
  }
  __syncthreads();
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  const uint64_t start = (uint64_t)b * bsize;
  const uint32_t len = (uint32_t)((n - start) < bsize ? (n - start) : bsize);
  const uint8_t* p = src + start;
  uint32_t c = 0xffffffffu, i = 0;
  auto word = [&](uint32_t w) {
    c ^= w;
    c = T[3][c & 0xff] ^ T[2][(c >> 8) & 0xff] ^ T[1][(c >> 16) & 0xff] ^ T[0][c >> 24];
  };
  if (((uintptr_t)p & 15u) == 0) {
    uint4 v = len >= 16 ? *(const uint4*)p : make_uint4(0, 0, 0, 0);
    for (; i + 16 <= len; i += 16) {
      const uint4 cur = v;
      if (i + 32 <= len) v = *(const uint4*)(p + i + 16);  // next quad in flight
      word(cur.x);
      word(cur.y);
      word(cur.z);
      word(cur.w);
    }
  }
  for (; i < len; ++i) c = T[0][(c ^ p[i]) & 0xffu] ^ (c >> 8);
  crc_out[b] = ~c;
}

}  // namespace hbam
