// Lane-occupancy model of the Huffman lane pass (k_inflate_tokens, inflate_tok.h) — tooling only.
//
// Walks every BGZF block of a BAM file, decodes its DEFLATE symbols (RFC 1951, a plain bit-serial
// canonical decoder) and counts, per DEFLATE block ("phase"), the symbol-loop iterations the lane
// pass spends on it: one iteration takes a literal and a second lit/len symbol, or a literal and a
// match, or a match (tok_fast_spec).  Output: one text line per BGZF block,
//   clen isize nphase it0 it1 ... (iterations per phase)
// tools/lane_sim.py folds these into waves of 64 lanes as the kernel runs them.
//
// usage: lane_sim FILE.bam [MAX_BLOCKS] > blocks.txt
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  const uint8_t* p;
  size_t n, pos;  // bit position
} Bits;
static uint32_t getbit(Bits* b) {
  const size_t i = b->pos >> 3;
  const uint32_t v = i < b->n ? (b->p[i] >> (b->pos & 7)) & 1u : 0u;
  ++b->pos;
  return v;
}
static uint32_t getbits(Bits* b, int k) {
  uint32_t v = 0;
  for (int i = 0; i < k; ++i) v |= getbit(b) << i;
  return v;
}
typedef struct {
  uint16_t cnt[16], sym[320];
} Huf;
static int build(Huf* h, const uint8_t* len, int n) {
  uint16_t offs[16];
  memset(h->cnt, 0, sizeof h->cnt);
  for (int s = 0; s < n; ++s) h->cnt[len[s]]++;
  h->cnt[0] = 0;
  offs[1] = 0;
  for (int l = 1; l < 15; ++l) offs[l + 1] = offs[l] + h->cnt[l];
  for (int s = 0; s < n; ++s)
    if (len[s]) h->sym[offs[len[s]]++] = (uint16_t)s;
  return 0;
}
static int decode(Bits* b, const Huf* h) {
  int code = 0, first = 0, index = 0;
  for (int l = 1; l < 16; ++l) {
    code |= (int)getbit(b);
    const int c = h->cnt[l];
    if (code - c < first) return h->sym[index + (code - first)];
    index += c;
    first += c;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}
static const uint16_t LB[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t LE[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint8_t DE[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

// one Huffman-coded DEFLATE block: iterations of the lane pass's symbol loop
static long phase(Bits* b, const Huf* ll, const Huf* d) {
  long it = 0;
  int pending_lit = 0;  // a literal already taken in the current iteration
  for (;;) {
    const int s = decode(b, ll);
    if (s < 0) return -1;
    if (s < 256) {
      if (pending_lit) {
        pending_lit = 0;  // second literal closes the iteration
      } else {
        pending_lit = 1;
        ++it;
      }
      continue;
    }
    if (s == 256) return it;
    if (!pending_lit) ++it;  // a match alone opens (and closes) an iteration
    pending_lit = 0;
    const int li = s - 257;
    if (li > 28) return -1;
    getbits(b, LE[li]);
    const int ds = decode(b, d);
    if (ds < 0 || ds > 29) return -1;
    getbits(b, DE[ds]);
  }
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  const long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* buf = (uint8_t*)malloc((size_t)sz);
  if (fread(buf, 1, (size_t)sz, f) != (size_t)sz) return 2;
  const long maxb = argc > 2 ? atol(argv[2]) : -1;
  static const uint8_t ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
  long o = 0, nb = 0;
  while (o + 18 <= sz && (maxb < 0 || nb < maxb)) {
    const uint32_t bsize = (uint32_t)(buf[o + 16] | buf[o + 17] << 8) + 1u;
    const uint32_t clen = bsize - 26u;
    const uint32_t isize = (uint32_t)(buf[o + bsize - 4] | buf[o + bsize - 3] << 8 | buf[o + bsize - 2] << 16 |
                                      (uint32_t)buf[o + bsize - 1] << 24);
    Bits b = {buf + o + 18, clen, 0};
    long its[64];
    int np = 0, last = 0;
    while (!last && np < 64) {
      last = (int)getbit(&b);
      const uint32_t type = getbits(&b, 2);
      uint8_t len[320];
      Huf ll, d;
      if (type == 0) {
        b.pos = (b.pos + 7) & ~(size_t)7;
        const uint32_t n = getbits(&b, 16);
        getbits(&b, 16);
        b.pos += 8 * (size_t)n;
        its[np++] = (long)(n + 1) / 2;
        continue;
      } else if (type == 1) {
        for (int s = 0; s < 288; ++s) len[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
        build(&ll, len, 288);
        for (int s = 0; s < 30; ++s) len[s] = 5;
        build(&d, len, 30);
      } else if (type == 2) {
        const int nlen = (int)getbits(&b, 5) + 257, ndist = (int)getbits(&b, 5) + 1, ncode = (int)getbits(&b, 4) + 4;
        uint8_t cl[19] = {0};
        for (int i = 0; i < ncode; ++i) cl[ord[i]] = (uint8_t)getbits(&b, 3);
        Huf hc;
        build(&hc, cl, 19);
        int have = 0;
        while (have < nlen + ndist) {
          const int s = decode(&b, &hc);
          if (s < 16) {
            len[have++] = (uint8_t)s;
          } else if (s == 16) {
            const int r = 3 + (int)getbits(&b, 2);
            const uint8_t pv = len[have - 1];
            for (int k = 0; k < r; ++k) len[have++] = pv;
          } else {
            const int r = s == 17 ? 3 + (int)getbits(&b, 3) : 11 + (int)getbits(&b, 7);
            for (int k = 0; k < r; ++k) len[have++] = 0;
          }
        }
        build(&ll, len, nlen);
        build(&d, len + nlen, ndist);
      } else {
        break;
      }
      its[np++] = phase(&b, &ll, &d);
    }
    printf("%u %u %d", clen, isize, np);
    for (int i = 0; i < np; ++i) printf(" %ld", its[i]);
    printf("\n");
    o += bsize;
    ++nb;
  }
  return 0;
}
