// sync_sim.c — CPU model of the self-synchronising wave-per-block Huffman pass (design study
// for k_inflate_sync, not the oracle).  For every BGZF block of a file: parse each DEFLATE
// block's header, build the two-level lookup tables the kernel builds (root ROOT_LL / ROOT_D
// bits, per-entry canonical construction), run phase 1 (64 lanes decode from equally spaced
// bit offsets, record the symbol starts of their first W bits, verify synchronisation with the
// next lane, count output bytes up to the hand-off point h) and phase 2 (each lane of the chain
// decodes [h_k, h_k+1) exactly), execute the tokens and compare the block with zlib's output.
// Reports the wave cost (max over lanes per phase) against the sequential symbol count.
//
//   gcc -O2 -o /tmp/sync_sim tools/sync_sim.c -lz && /tmp/sync_sim FILE.bam [W] [SEGMIN] [LANES]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#define ROOT_LL 10
#define ROOT_D 8
#define CAP_LL 2048
#define CAP_D 512

static const uint16_t LBASE[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59,
                                   67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t DBASE[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                   1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t DEXT[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

static const uint8_t* g_data;
static uint32_t g_nbits;

static uint32_t peek(uint32_t pos, int n) {  // n <= 32, zero beyond the end
  uint64_t v = 0;
  uint32_t byte = pos >> 3;
  for (int i = 0; i < 6; ++i) {
    uint32_t b = byte + i;
    uint64_t x = (b < (g_nbits >> 3)) ? g_data[b] : 0;
    v |= x << (8 * i);
  }
  v >>= (pos & 7);
  return (uint32_t)(v & ((n == 32) ? 0xffffffffull : ((1ull << n) - 1)));
}
static uint32_t rev(uint32_t x, int n) {
  uint32_t r = 0;
  for (int i = 0; i < n; ++i) r |= ((x >> i) & 1u) << (n - 1 - i);
  return r;
}

typedef struct {
  uint16_t e[CAP_LL];
  int root, used, maxl;
} Lut;
// entry: direct sym | len << 9 (len 0 = no code); pointer 0x8000 | sb << 11 | off
static int lut_build(Lut* t, const uint8_t* lens, int n, int root, int cap, int* nlong) {
  int cnt[16] = {0}, fc[16] = {0}, offs[16] = {0};
  uint16_t sorted[288];
  for (int s = 0; s < n; ++s) cnt[lens[s]]++;
  cnt[0] = 0;
  int code = 0, maxl = 0;
  for (int l = 1; l < 16; ++l) {
    fc[l] = code;
    code = (code + cnt[l]) << 1;
    if (cnt[l]) maxl = l;
  }
  int o = 0;
  for (int l = 1; l < 16; ++l) {
    offs[l] = o;
    o += cnt[l];
  }
  int nx[16];
  memcpy(nx, offs, sizeof nx);
  for (int s = 0; s < n; ++s)
    if (lens[s]) sorted[nx[lens[s]]++] = (uint16_t)s;
  t->root = root;
  t->maxl = maxl;
  int used = 1 << root;
  *nlong = 0;
  for (int i = 0; i < (1 << root); ++i) {
    const uint32_t v = rev((uint32_t)i, root);
    uint16_t ent = 0;
    for (int l = 1; l <= root && l <= 15; ++l) {
      const uint32_t c = v >> (root - l);
      if (cnt[l] && c - (uint32_t)fc[l] < (uint32_t)cnt[l]) {
        ent = (uint16_t)(sorted[offs[l] + c - fc[l]] | l << 9);
        break;
      }
    }
    if (!ent) {  // longest code under prefix v
      int ml = 0;
      for (int l = root + 1; l <= maxl; ++l) {
        if (!cnt[l]) continue;
        const uint32_t lo = (uint32_t)fc[l] >> (l - root), hi = (uint32_t)(fc[l] + cnt[l] - 1) >> (l - root);
        if (v >= lo && v <= hi) ml = l;
      }
      if (ml) {
        const int sb = ml - root;
        if (used + (1 << sb) > cap) return -1;
        ent = (uint16_t)(0x8000 | sb << 11 | used);
        for (int j = 0; j < (1 << sb); ++j) {
          const uint32_t full = v << sb | rev((uint32_t)j, sb);
          uint16_t se = 0;
          for (int l = root + 1; l <= root + sb; ++l) {
            const uint32_t c = full >> (root + sb - l);
            if (cnt[l] && c - (uint32_t)fc[l] < (uint32_t)cnt[l]) {
              se = (uint16_t)(sorted[offs[l] + c - fc[l]] | l << 9);
              break;
            }
          }
          t->e[used + j] = se;
        }
        used += 1 << sb;
        ++*nlong;
      }
    }
    t->e[i] = ent;
  }
  t->used = used;
  return 0;
}
static uint16_t lut_get(const Lut* t, uint32_t pos) {
  uint16_t e = t->e[peek(pos, t->root)];
  if (e & 0x8000) {
    const int sb = (e >> 11) & 15;
    e = t->e[(e & 0x7ff) + (peek(pos, t->root + sb) >> t->root)];
  }
  return e;
}

enum { S_LIT, S_MATCH, S_EOB, S_BAD };
typedef struct {
  int kind;
  uint32_t bits, out, lit, dist;
} Sym;
static Sym decode(const Lut* ll, const Lut* d, uint32_t pos) {
  Sym s = {S_BAD, 1, 1, 0, 0};
  const uint16_t e = lut_get(ll, pos);
  const uint32_t l = (e >> 9) & 15, sym = e & 511;
  if (!l) return s;  // spec: 1 bit, 1 byte
  if (sym < 256) {
    s.kind = S_LIT, s.bits = l, s.out = 1, s.lit = sym;
    return s;
  }
  if (sym == 256) {
    s.kind = S_EOB, s.bits = l, s.out = 0;
    return s;
  }
  s.bits = l;
  if (sym > 285) return s;
  const uint32_t li = sym - 257;
  const uint32_t mlen = LBASE[li] + peek(pos + l, LEXT[li]);
  uint32_t p = pos + l + LEXT[li];
  const uint16_t de = lut_get(d, p);
  const uint32_t dl = (de >> 9) & 15, ds = de & 511;
  if (!dl || ds > 29) {
    s.bits = p - pos + (dl ? dl : 1);
    return s;
  }
  p += dl;
  const uint32_t dist = DBASE[ds] + peek(p, DEXT[ds]);
  p += DEXT[ds];
  s.kind = S_MATCH, s.bits = p - pos, s.out = mlen, s.dist = dist;
  return s;
}

static int g_W = 640, g_SEGMIN = 1280, g_LANES = 64;
static uint64_t st_blocks, st_dblocks, st_fallback, st_syms, st_wave1, st_wave2, st_mism, st_nosync,
    st_bigtab, st_long_ll, st_long_d, st_lanes, st_hdrsyms;
static uint64_t st_fb_reason[8];

// one DEFLATE block's symbols from `start`; out/op: output so far. Returns end bit (after EOB) or ~0 on fallback
static uint32_t sync_block(const Lut* ll, const Lut* d, uint32_t start, uint8_t* out, uint32_t* op, uint32_t isize) {
  const uint32_t end = g_nbits;
  uint32_t span = end > start ? end - start : 0;
  uint32_t seg = (span + g_LANES - 1) / g_LANES;
  if (seg < (uint32_t)g_SEGMIN) seg = g_SEGMIN;
  int L = (int)((span + seg - 1) / seg);
  if (L < 1) L = 1;
  if (L > 64) L = 64;
  st_lanes += L;
  static uint8_t bm[64][4096];
  uint32_t s[65], h[65], cnt_h[65], cnt_end[65], stop[65], eob[65];
  int status[65];  // 0 sync, 1 nosync, 2 eob, 3 runout
  uint32_t it1[65];
  for (int k = 0; k < L; ++k) s[k] = start + (uint32_t)k * seg;
  // bitmaps first (the kernel's lanes write theirs before anyone checks)
  for (int k = 0; k < L; ++k) {
    memset(bm[k], 0, (g_W + 7) / 8);
    uint32_t x = s[k];
    while (x < s[k] + g_W) {
      bm[k][(x - s[k]) >> 3] |= 1u << ((x - s[k]) & 7);
      Sym y = decode(ll, d, x);
      x += y.bits;
    }
  }
  for (int k = 0; k < L; ++k) {
    uint32_t x = s[k], c = 0, it = 0;
    int synced = 0, hset = (k == 0);
    h[k] = start;
    cnt_h[k] = 0;
    status[k] = 3;
    for (;;) {
      if (!hset && x >= s[k] + g_W) {
        h[k] = x, cnt_h[k] = c, hset = 1;
      }
      if (k + 1 < L) {
        if (x >= s[k + 1] + g_W) {
          status[k] = synced ? 0 : 1;
          break;
        }
        if (x >= s[k + 1] && (bm[k + 1][(x - s[k + 1]) >> 3] >> ((x - s[k + 1]) & 7) & 1)) synced = 1;
      }
      if (x >= end) {
        status[k] = 3;
        break;
      }
      Sym y = decode(ll, d, x);
      if (hset && y.kind == S_EOB) {
        status[k] = 2;
        eob[k] = x + y.bits;
        break;
      }
      x += y.bits;
      c += y.out;
      ++it;
    }
    stop[k] = x;
    cnt_end[k] = c;
    it1[k] = it;
  }
  uint32_t w1 = 0;
  for (int k = 0; k < L; ++k) w1 = it1[k] > w1 ? it1[k] : w1;
  st_wave1 += w1;
  int owner = -1;
  for (int k = 0; k < L; ++k) {
    if (status[k] == 2) {
      owner = k;
      break;
    }
    if (status[k] != 0) {
      if (status[k] == 1) ++st_nosync;
      st_fb_reason[status[k] == 1 ? 1 : 2]++;
      return ~0u;
    }
  }
  if (owner < 0) {
    st_fb_reason[3]++;
    return ~0u;
  }
  // phase 2: exact decode of each chain lane's portion
  uint32_t w2 = 0, o = *op;
  for (int k = 0; k <= owner; ++k) {
    const uint32_t a = h[k], b = (k == owner) ? eob[k] : h[k + 1];
    uint32_t x = a, it = 0;
    const uint32_t want = (k == owner ? cnt_end[k] : cnt_end[k]) - cnt_h[k];
    uint32_t got = 0;
    for (;;) {
      if (k != owner && x >= b) break;
      Sym y = decode(ll, d, x);
      if (y.kind == S_EOB) {
        if (k != owner || x + y.bits != b) {
          st_fb_reason[4]++;
          return ~0u;
        }
        break;
      }
      if (y.kind == S_BAD) {
        st_fb_reason[5]++;
        return ~0u;
      }
      if (o + y.out > isize) {
        st_fb_reason[6]++;
        return ~0u;
      }
      if (y.kind == S_LIT) {
        out[o++] = (uint8_t)y.lit;
      } else {
        if (y.dist > o) {
          st_fb_reason[7]++;
          return ~0u;
        }
        for (uint32_t j = 0; j < y.out; ++j, ++o) out[o] = out[o - y.dist];
      }
      got += y.out;
      x += y.bits;
      ++it;
    }
    if (got != want) {
      fprintf(stderr, "count mismatch lane %d: %u vs %u\n", k, got, want);
      exit(2);
    }
    w2 = it > w2 ? it : w2;
    st_syms += it;
  }
  st_wave2 += w2;
  *op = o;
  return eob[owner];
}

static const uint8_t ORD[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// returns 0 ok (matches zlib), 1 fallback
static int run_block(const uint8_t* cdata, uint32_t nbytes, uint32_t isize, uint8_t* out, const uint8_t* ref) {
  g_data = cdata;
  g_nbits = nbytes * 8;
  uint32_t pos = 0, op = 0;
  for (;;) {
    const uint32_t fin = peek(pos, 1), type = peek(pos + 1, 2);
    pos += 3;
    uint8_t lens[320];
    int nlen, ndist;
    if (type == 1) {
      for (int s = 0; s < 288; ++s) lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
      for (int s = 0; s < 32; ++s) lens[288 + s] = 5;
      nlen = 288, ndist = 32;
    } else if (type == 2) {
      nlen = (int)peek(pos, 5) + 257, ndist = (int)peek(pos + 5, 5) + 1;
      const int ncode = (int)peek(pos + 10, 4) + 4;
      pos += 14;
      uint8_t cl[19] = {0};
      for (int i = 0; i < ncode; ++i, pos += 3) cl[ORD[i]] = (uint8_t)peek(pos, 3);
      Lut tc;
      int nl;
      if (lut_build(&tc, cl, 19, 7, CAP_LL, &nl)) return 1;
      uint8_t all[320];
      int have = 0;
      while (have < nlen + ndist) {
        const uint16_t e = lut_get(&tc, pos);
        const uint32_t l = (e >> 9) & 15, sym = e & 511;
        if (!l) return 1;
        pos += l;
        st_hdrsyms++;
        if (sym < 16) {
          all[have++] = (uint8_t)sym;
        } else {
          uint32_t rep, v = 0;
          if (sym == 16) {
            if (!have) return 1;
            v = all[have - 1], rep = 3 + peek(pos, 2), pos += 2;
          } else if (sym == 17) {
            rep = 3 + peek(pos, 3), pos += 3;
          } else {
            rep = 11 + peek(pos, 7), pos += 7;
          }
          if (have + (int)rep > nlen + ndist) return 1;
          while (rep--) all[have++] = (uint8_t)v;
        }
      }
      memcpy(lens, all, nlen);
      memset(lens + nlen, 0, 288 - nlen);
      memcpy(lens + 288, all + nlen, ndist);
      memset(lens + 288 + ndist, 0, 32 - ndist);
    } else {
      st_fb_reason[0]++;
      return 1;
    }
    st_dblocks++;
    static Lut ll, dd;
    int nl1, nl2;
    if (lut_build(&ll, lens, 288, ROOT_LL, CAP_LL, &nl1) || lut_build(&dd, lens + 288, 32, ROOT_D, CAP_D, &nl2)) {
      st_bigtab++;
      return 1;
    }
    st_long_ll += nl1;
    st_long_d += nl2;
    const uint32_t e = sync_block(&ll, &dd, pos, out, &op, isize);
    if (e == ~0u) return 1;
    pos = e;
    if (fin) break;
  }
  if (op != isize || pos > g_nbits) return 1;
  if (memcmp(out, ref, isize)) {
    ++st_mism;
    return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) return 1;
  if (argc > 2) g_W = atoi(argv[2]);
  if (argc > 3) g_SEGMIN = atoi(argv[3]);
  if (argc > 4) g_LANES = atoi(argv[4]);
  FILE* f = fopen(argv[1], "rb");
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* buf = malloc(n);
  if (fread(buf, 1, n, f) != (size_t)n) return 1;
  fclose(f);
  static uint8_t out[65536], ref[65536];
  long p = 0;
  while (p + 18 <= n) {
    const uint32_t bsize = (uint32_t)(buf[p + 16] | buf[p + 17] << 8) + 1;
    const uint8_t* cd = buf + p + 18;
    const uint32_t clen = bsize - 26;
    const uint32_t isize = buf[p + bsize - 4] | buf[p + bsize - 3] << 8 | buf[p + bsize - 2] << 16 |
                           (uint32_t)buf[p + bsize - 1] << 24;
    z_stream z;
    memset(&z, 0, sizeof z);
    inflateInit2(&z, -15);
    z.next_in = (uint8_t*)cd, z.avail_in = clen, z.next_out = ref, z.avail_out = isize;
    inflate(&z, Z_FINISH);
    inflateEnd(&z);
    st_blocks++;
    if (isize && run_block(cd, clen, isize, out, ref)) st_fallback++;
    p += bsize;
  }
  printf("W %d segmin %d lanes %d: blocks %lu deflate-blocks %lu fallback %lu (mismatch %lu, nosync %lu, bigtab %lu)"
         " reasons %lu %lu %lu %lu %lu %lu %lu %lu\n",
         g_W, g_SEGMIN, g_LANES, st_blocks, st_dblocks, st_fallback, st_mism, st_nosync, st_bigtab, st_fb_reason[0],
         st_fb_reason[1], st_fb_reason[2], st_fb_reason[3], st_fb_reason[4], st_fb_reason[5], st_fb_reason[6],
         st_fb_reason[7]);
  printf("symbols/block %.0f  header syms/block %.1f  wave iters/block: phase1 %.0f phase2 %.0f total %.0f"
         "  (%.3f of sequential/64)  lanes/dblock %.1f  long prefixes/dblock ll %.1f d %.1f\n",
         (double)st_syms / st_blocks, (double)st_hdrsyms / st_blocks, (double)st_wave1 / st_blocks,
         (double)st_wave2 / st_blocks, (double)(st_wave1 + st_wave2) / st_blocks,
         (double)(st_wave1 + st_wave2) / ((double)st_syms / 64.0), (double)st_lanes / st_dblocks,
         (double)st_long_ll / st_dblocks, (double)st_long_d / st_dblocks);
  return 0;
}
