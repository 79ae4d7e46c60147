// CPU model of ONE lane of k_inflate_tokens (inflate_tok.h) for MemorySanitizer: every BGZF block
// of a blocks file (tools/cpu_model/make_blocks.py) is decoded by the unmodified per-lane
// function `inflate_tokens_block` into its token form (literals, 3-byte match descriptors, match-
// start bitmap, tail token, edge slots), the edge slots are merged as k_edge_merge does, the
// tokens are resolved by a sequential restatement of k_resolve's contract, and the bytes are
// compared with zlib's (the file's expected bytes).
//
// What the GPU leaves stale is left uninitialised here: the per-lane LDS symbol tables, the
// code-length scratch, the bitmap, the tail slot, the edge slots and the output chunks are
// malloc'd fresh per block and never cleared, so a read of a slot the decode has not written that
// reaches a branch, an address or the compared output is reported by MSan with its origin.
// Built by tools/cpu_model/build.py; tests/test_cpu_model.py runs it.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "inflate_tok.h"

using namespace hbam;

static constexpr uint32_t LENS_SLOT_M = 352;      // hbam_internal.h LENS_SLOT
static constexpr uint32_t BITMAP_WORDS_M = 2048;  // hbam_internal.h BITMAP_WORDS

static void* xalloc(size_t n) {  // 16-aligned, uninitialised
  void* p = aligned_alloc(16, (n + 15) & ~(size_t)15);
  if (!p) {
    fprintf(stderr, "out of memory\n");
    exit(3);
  }
  return p;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s blocks.bin\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) {
    perror(argv[1]);
    return 2;
  }
  uint32_t hdr[2];
  if (fread(hdr, 4, 2, f) != 2 || hdr[0] != 0x4d544248u) {  // "HBTM"
    fprintf(stderr, "bad blocks file\n");
    return 2;
  }
  const uint32_t n = hdr[1];
  uint32_t bad = 0, short_ = 0, data = 0;
  uint64_t ubytes = 0;
  for (uint32_t b = 0; b < n; ++b) {
    uint32_t m[2];
    if (fread(m, 4, 2, f) != 2) return 2;
    const uint32_t clen = m[0], isize = m[1];
    // compressed bytes as on the device: inside the file, over-reads of up to two quads past the
    // stream land on initialised bytes (the next block / the 64-byte zero pad)
    const uint32_t a = b & 15u;
    uint8_t* cbuf = (uint8_t*)xalloc(a + clen + 96);
    memset(cbuf, 0, a + clen + 96);
    uint8_t* expect = (uint8_t*)malloc(isize ? isize : 1);
    if (fread(cbuf + a, 1, clen, f) != clen || fread(expect, 1, isize, f) != isize) return 2;
    // stale on the GPU: LDS tables, length scratch, bitmap, tail, edge slots, output chunks
    uint8_t* syms_ll = (uint8_t*)xalloc(288);
    uint8_t* syms_d = (uint8_t*)xalloc(32);
    uint8_t* lens = (uint8_t*)xalloc(LENS_SLOT_M);
    uint32_t* bm = (uint32_t*)xalloc(4 * BITMAP_WORDS_M);
    uint32_t* tails = (uint32_t*)xalloc(8);
    uint8_t* edge = (uint8_t*)xalloc(32);
    const uint32_t start = (b * 7u) & 15u;  // every output misalignment occurs
    uint8_t* ubuf = (uint8_t*)xalloc(start + isize + 32);
#ifdef HBAM_MODEL_SELFTEST
    // negative control (tests/test_cpu_model.py): a stale symbol slot read into a branch
    if (syms_ll[5] == 7u) puts("stale slot");
#endif
    TSink sink;
    sink.init(ubuf, start, isize, bm, tails, edge);
    uint32_t produced = 0;
#ifdef HBAM_PROF
    uint64_t pt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pc[4] = {0, 0, 0, 0};
#endif
    const int32_t rc = inflate_tokens_block(cbuf + a, clen, isize, syms_ll, syms_d, lens, sink, &produced
#ifdef HBAM_PROF
                                            , pt, pc
#endif
    );
    bool ok = rc == INF_OK && produced == isize;
    if (rc == INF_SHORT) ++short_;
    if (rc == INF_DATA) ++data;
    if (ok && isize) {
      // k_edge_merge (hbam_kernels.hip): the partial first / last chunk from the edge slots
      const uint32_t soff = start, iend = soff + isize;
      if (soff != 0) {
        const uint32_t hi = iend < 16u ? iend : 16u;
        for (uint32_t r = soff; r < hi; ++r) ubuf[r] = edge[r & 15u];
      }
      const uint32_t cl = (iend - 1u) >> 4;
      if (!((iend & 15u) == 0 || (cl == 0 && soff != 0)))
        for (uint32_t r = cl << 4; r < iend; ++r) ubuf[r] = edge[16u + (r & 15u)];
      // k_resolve's contract, sequentially: a set bitmap bit at p = a descriptor (len-3, dist-1)
      // in the first 3 bytes of the match at p; then the optional short final match
      uint8_t* out = ubuf + soff;
      for (uint32_t p = 0; p < isize && ok;) {
        const uint32_t w = (p >> 7) * 4u + ((p & 127u) >> 5);
        if ((bm[w] >> (p & 31u)) & 1u) {
          const uint32_t len = out[p] + 3u, dist = (out[p + 1] | (uint32_t)out[p + 2] << 8) + 1u;
          if (dist > p || p + len > isize) {
            ok = false;
            break;
          }
          for (uint32_t k = 0; k < len; ++k) out[p + k] = out[p + k - dist];
          p += len;
        } else {
          ++p;
        }
      }
      if (ok && (tails[0] & 0x80000000u)) {
        const uint32_t p = tails[0] & 0xffffu, nn = (tails[0] >> 16) & 0x7fffu, d = tails[1];
        if (d == 0 || d > p || p + nn > isize) ok = false;
        for (uint32_t k = 0; ok && k < nn; ++k) out[p + k] = out[p + k - d];
      }
      if (ok && memcmp(out, expect, isize) != 0) ok = false;
    }
    if (!ok) {
      ++bad;
      if (bad <= 10) fprintf(stderr, "block %u: rc %d produced %u isize %u: mismatch\n", b, rc, produced, isize);
    }
    ubytes += isize;
    free(cbuf);
    free(expect);
    free(syms_ll);
    free(syms_d);
    free(lens);
    free(bm);
    free(tails);
    free(edge);
    free(ubuf);
  }
  printf("blocks %u bytes %llu bad %u (short %u, data error %u)\n", n, (unsigned long long)ubytes, bad, short_, data);
  return bad ? 1 : 0;
}
