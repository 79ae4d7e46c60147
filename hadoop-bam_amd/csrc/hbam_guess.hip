// hbam_guess.hip — BAMSplitGuesser / BGZFSplitGuesser on the device (gfx950).
//
// One wave = one guesser call guessNextBAMRecordStart(beg, end) (BAMSplitGuesser.java:109-212),
// so BAMInputFormat.addProbabilisticSplits' per-split loop (BAMInputFormat.java:181-222) and
// config #3's 10k guesses run as one launch.  The wave runs the reference's state machine
// over the window W = file[beg, beg+min(end-beg, 262139)) with the same cursor semantics the
// Java code observes.  Kernels see each guess's window only (the bytes BAMSplitGuesser.java:
// 114-125 reads): wptr[i] = device address of file byte beg[i] (a view into a device-resident
// file, or the window a caller gathered), wlen[i] = bytes available there:
//   * SeekableArrayStream (util/SeekableArrayStream.java:29-58) — one shared position used by
//     both guessNextBGZFPos and the BlockCompressedInputStream, seek bounds, short reads;
//   * the persistent 8-byte ByteBuffer `buf` (stale bytes survive short reads);
//   * [htsjdk] BlockCompressedInputStream readBlock/available/read/seek/getFilePointer/eof
//     with CRC checking on (BAMSplitGuesser.java:130), block cache on seek;
//   * [htsjdk] BAMRecordCodec.decode with LazyBAMRecordFactory (no refID validation);
//   * the exception filter of :144-152 and :194-207.
// Inflate + CRC32 come from a per-window block cache: before the state machines run, every
// position of a window that carries the gzip magic is treated as a candidate block and
// inflated by the batched two-phase inflater (k_inflate_tokens + k_resolve, zlib-exact) with
// k_crc32, so a lane's readBlock is a binary search + a pointer, not a 64 KiB inflate.  A
// block the cache does not hold (candidate overflow, ISIZE > 65536) is inflated in-lane
// (inflate_dev.h, same contract).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbam_internal.h"
#include "inflate_dev.h"

namespace hbam {

constexpr int32_t G_MAGIC = 0x04088b1f;
constexpr int32_t G_MAGIC_SUB = 0x00024342;
constexpr int32_t G_MAX_BYTES_READ = 3 * 0xffff + 0xfffe;
constexpr uint32_t GUESS_WG = 64;
constexpr uint32_t GC_CAP = 256;      // cached candidate blocks per guess window

// Candidate blocks of one guess window (sorted absolute file offsets) and their inflated
// bytes / status / CRC in the batched-inflate buffers.
struct GCache {
  const uint64_t* pos;   // this window's candidates (n of them)
  uint32_t n;
  const BlockRec* blk;   // same indexing as pos
  const uint64_t* uoff;
  const uint8_t* ubuf;
  const int32_t* st;
  const uint32_t* crc;
};

struct GStream {  // SeekableArrayStream over the window
  const uint8_t* a;
  int64_t len;
  int64_t pos;
};
__device__ __forceinline__ bool gs_seek(GStream& s, int64_t p) {
  if (p < 0 || p > s.len) return false;  // IOException
  s.pos = p;
  return true;
}
__device__ __forceinline__ int32_t gs_read(GStream& s, uint8_t* b, int32_t n) {
  if (s.pos == s.len) return -1;
  if ((int64_t)n > s.len - s.pos) n = (int32_t)(s.len - s.pos);
  for (int32_t i = 0; i < n; ++i) b[i] = s.a[s.pos + i];
  s.pos += n;
  return n;
}

struct GBcis {
  int64_t block_addr;
  int32_t last_len;
  int32_t cur_len;  // -1 = mCurrentBlock == null
  int32_t cur_off;
  const uint8_t* cur;  // current block's inflated bytes (cache or scratch)
  uint8_t* scratch;    // 65536-byte global scratch for in-lane inflates
  int64_t wbase;       // absolute file offset of the window start
  GCache cache;        // cache.n == 0: no cache
  uint16_t* s_ll;
  uint8_t* s_d;
  uint8_t* lens;
  const uint32_t* crc_tab;
  int check_crc;
};

__device__ int32_t gb_read_block(GBcis& b, GStream& f) {
  const int64_t P = f.pos;
  const int64_t avail = f.len - P;
  if (avail <= 0) {  // count == 0: no empty gzip block at end
    b.cur_off = 0;
    b.block_addr += b.last_len;
    b.cur_len = 0;
    return HBAM_OK;
  }
  if (avail < 18) { f.pos = f.len; return HBAM_EIO; }  // Premature end of file
  const uint8_t* h = f.a + P;
  const int32_t blen = (int32_t)(h[16] | h[17] << 8) + 1;
  if (blen < 18) { f.pos = P + 18; return HBAM_EIO; }
  if ((int64_t)blen > avail) { f.pos = f.len; return HBAM_ETRUNC; }
  f.pos = P + blen;
  // inflateBlock: mCurrentBlock = null first
  b.cur_len = -1;
  const int32_t isize = (int32_t)((uint32_t)h[blen - 4] | (uint32_t)h[blen - 3] << 8 |
                                  (uint32_t)h[blen - 2] << 16 | (uint32_t)h[blen - 1] << 24);
  if (isize < 0) return HBAM_ERUNTIMEIO;
  // BlockGunzipper header checks
  if (!(h[0] == 0x1f && h[1] == 0x8b && h[2] == 8 && h[3] == 4)) return HBAM_EFORMAT;
  if ((h[10] | h[11] << 8) != 6) return HBAM_EFORMAT;
  if (blen < 26) return HBAM_EDATA;
  if (isize > 65536) return HBAM_EUNSUPPORTED;
  const uint32_t expect = (uint32_t)h[blen - 8] | (uint32_t)h[blen - 7] << 8 |
                          (uint32_t)h[blen - 6] << 16 | (uint32_t)h[blen - 5] << 24;
  // cache lookup (binary search over the window's sorted candidates)
  int32_t hit = -1;
  if (b.cache.n) {
    const uint64_t want = (uint64_t)(b.wbase + P);
    uint32_t lo = 0, hi = b.cache.n;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (b.cache.pos[mid] < want) lo = mid + 1; else hi = mid;
    }
    if (lo < b.cache.n && b.cache.pos[lo] == want && b.cache.blk[lo].pad &&
        b.cache.blk[lo].clen == (uint32_t)blen && b.cache.blk[lo].isize == (uint32_t)isize)
      hit = (int32_t)lo;
  }
  if (hit >= 0) {
    const int32_t st = b.cache.st[hit];
    if (st == INF_DATA) return HBAM_EDATA;
    if (st == INF_SHORT) return HBAM_EFORMAT;
    if (b.check_crc && b.cache.crc[hit] != expect) return HBAM_EFORMAT;
    b.cur = b.cache.ubuf + b.cache.uoff[hit];
  } else {
    uint32_t produced = 0;
    const int32_t st = inflate_raw(h + 18, (uint32_t)(blen - 26), b.scratch, (uint32_t)isize, b.s_ll,
                                   b.s_d, b.lens, &produced);
    if (st == INF_DATA) return HBAM_EDATA;
    if (st == INF_SHORT) return HBAM_EFORMAT;
    if (b.check_crc) {
      uint32_t c = 0xffffffffu;
      for (int32_t i = 0; i < isize; ++i) c = b.crc_tab[(c ^ b.scratch[i]) & 0xff] ^ (c >> 8);
      if (~c != expect) return HBAM_EFORMAT;
    }
    b.cur = b.scratch;
  }
  b.cur_len = isize;
  b.cur_off = 0;
  b.block_addr += b.last_len;
  b.last_len = blen;
  return HBAM_OK;
}
__device__ int32_t gb_available(GBcis& b, GStream& f, int32_t* avail) {
  if (b.cur_len < 0 || b.cur_off == b.cur_len) {
    const int32_t rc = gb_read_block(b, f);
    if (rc) return rc;
  }
  *avail = b.cur_len < 0 ? 0 : b.cur_len - b.cur_off;
  return HBAM_OK;
}
// read(): copy into dst (or skip when dst == nullptr); *got = -1 at EOF
__device__ int32_t gb_read(GBcis& b, GStream& f, uint8_t* dst, int32_t len, int32_t* got) {
  const int32_t orig = len;
  int32_t off = 0;
  while (len > 0) {
    int32_t av;
    const int32_t rc = gb_available(b, f, &av);
    if (rc) return rc;
    if (av == 0) {
      if (orig == len) { *got = -1; return HBAM_OK; }
      break;
    }
    const int32_t c = len < av ? len : av;
    if (dst)
      for (int32_t i = 0; i < c; ++i) dst[off + i] = b.cur[b.cur_off + i];
    b.cur_off += c;
    off += c;
    len -= c;
  }
  *got = orig - len;
  return HBAM_OK;
}
__device__ __forceinline__ bool gb_eof(const GBcis& b, const GStream& f) {
  if (f.pos == f.len) return true;
  return f.len - (b.block_addr + b.last_len) == 28;
}
__device__ int32_t gb_seek(GBcis& b, GStream& f, uint64_t pos) {
  const int64_t coff = (int64_t)(pos >> 16);
  const int32_t uoff = (int32_t)(pos & 0xffff);
  int32_t avail;
  if (b.block_addr == coff && b.cur_len >= 0) {
    avail = b.cur_len;
  } else {
    if (!gs_seek(f, coff)) return HBAM_EIO;
    b.block_addr = coff;
    b.last_len = 0;
    int32_t rc = gb_read_block(b, f);
    if (rc) return rc;
    rc = gb_available(b, f, &avail);
    if (rc) return rc;
  }
  if (uoff > avail || (uoff == avail && !gb_eof(b, f))) return HBAM_EIO;
  b.cur_off = uoff;
  return HBAM_OK;
}
__device__ __forceinline__ uint64_t gb_tell(const GBcis& b) {
  if (b.cur_off == b.cur_len) return (uint64_t)(b.block_addr + b.last_len) << 16;
  return (uint64_t)b.block_addr << 16 | (uint32_t)b.cur_off;
}
// BinaryCodec.readBytes: IOException -> RuntimeIOException, -1 -> RuntimeEOFException
__device__ int32_t gc_read(GBcis& b, GStream& f, uint8_t* dst, int32_t len) {
  int32_t total = 0;
  do {
    int32_t got;
    int32_t rc = gb_read(b, f, dst ? dst + total : nullptr, len - total, &got);
    if (rc == HBAM_EIO) return HBAM_ERUNTIMEIO;
    if (rc) return rc;
    if (got < 0) return HBAM_EEOF;
    total += got;
  } while (total < len);
  return HBAM_OK;
}
// BAMRecordCodec.decode with the lazy factory: 1 record, 0 null, <0 exception
__device__ int32_t gc_decode(GBcis& b, GStream& f) {
  // whole record inside the current block: the reads below only advance cur_off
  if (b.cur_len >= 0 && b.cur_len - b.cur_off >= 4) {
    const uint8_t* q = b.cur + b.cur_off;
    const int32_t bs = (int32_t)((uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 |
                                 (uint32_t)q[3] << 24);
    if (bs < 32) {
      b.cur_off += 4;
      return HBAM_EFORMAT;
    }
    if (b.cur_len - b.cur_off - 4 >= bs) {
      b.cur_off += 4 + bs;
      return 1;
    }
  }
  uint8_t t[4];
  int32_t rc = gc_read(b, f, t, 4);
  if (rc == HBAM_EEOF) return 0;
  if (rc) return rc;
  const int32_t bs = (int32_t)((uint32_t)t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 |
                               (uint32_t)t[3] << 24);
  if (bs < 32) return HBAM_EFORMAT;
  const int32_t fields[11] = {4, 4, 1, 1, 2, 2, 2, 4, 4, 4, 4};
#pragma unroll
  for (int k = 0; k < 11; ++k) {
    rc = gc_read(b, f, nullptr, fields[k]);
    if (rc) return rc;
  }
  if (bs > 32) {
    rc = gc_read(b, f, nullptr, bs - 32);
    if (rc) return rc;
  }
  return 1;
}

struct Guesser {
  GStream in;
  GBcis bz;
  uint8_t buf[8];
  int32_t n_ref;
};
__device__ __forceinline__ int32_t gbuf_i32(const Guesser& g, int i) {
  return (int32_t)((uint32_t)g.buf[i] | (uint32_t)g.buf[i + 1] << 8 | (uint32_t)g.buf[i + 2] << 16 |
                   (uint32_t)g.buf[i + 3] << 24);
}
__device__ __forceinline__ int32_t gbuf_u16(const Guesser& g, int i) {
  return (int32_t)(g.buf[i] | g.buf[i + 1] << 8);
}

// guessNextBGZFPos :222-299 (IOException -> null)
__device__ bool g_next_bgzf(Guesser& g, int32_t p, int32_t end, int32_t* opos, int32_t* osize) {
  for (;;) {
    for (;;) {
      if (!gs_seek(g.in, p)) return false;
      gs_read(g.in, g.buf, 4);
      const int32_t n = gbuf_i32(g, 0);
      if (n == G_MAGIC) break;
      if ((int32_t)((uint32_t)n >> 8) == 0x00088b1f) ++p;
      else if ((int32_t)((uint32_t)n >> 16) == 0x00008b1f) p += 2;
      else p += 3;
      if (p >= end) return false;
    }
    const int32_t p0 = p;
    p += 10;
    if (!gs_seek(g.in, p)) return false;
    gs_read(g.in, g.buf, 2);
    p += 2;
    const int32_t xlen = gbuf_u16(g, 0);
    const int32_t sub_end = p + xlen;
    bool cancel = false;
    while (p < sub_end) {
      gs_read(g.in, g.buf, 4);
      if (gbuf_i32(g, 0) != G_MAGIC_SUB) {
        p += 4 + gbuf_u16(g, 2);
        if (!gs_seek(g.in, p)) return false;
        continue;
      }
      gs_read(g.in, g.buf, 2);
      const int32_t bsize = gbuf_u16(g, 0);
      p += 6;
      while (p < sub_end) {
        if (!gs_seek(g.in, p)) return false;
        gs_read(g.in, g.buf, 4);
        p += 4 + gbuf_u16(g, 2);
      }
      if (p != sub_end) { cancel = true; break; }
      p += bsize - xlen - 19 + 4;
      if (!gs_seek(g.in, p)) return false;
      gs_read(g.in, g.buf, 4);
      *opos = p0;
      *osize = gbuf_i32(g, 0);
      return true;
    }
    (void)cancel;
    p = p0 + 4;
  }
}

// guessNextBAMPos :301-398
__device__ int32_t g_next_bam(Guesser& g, uint64_t cpv, int32_t up, int32_t csize) {
  int32_t got;
  up += 4;
  while (up + 35 < csize) {
    if (gb_seek(g.bz, g.in, cpv | (uint32_t)up)) return -1;
    if (gb_read(g.bz, g.in, g.buf, 8, &got)) return -1;
    const int32_t id = gbuf_i32(g, 0), pos = gbuf_i32(g, 4);
    if (id < -1 || id > g.n_ref || pos < -1) { ++up; continue; }
    if (gb_seek(g.bz, g.in, cpv | (uint32_t)(up + 20))) return -1;
    if (gb_read(g.bz, g.in, g.buf, 8, &got)) return -1;
    const int32_t nid = gbuf_i32(g, 0), npos = gbuf_i32(g, 4);
    if (nid < -1 || nid > g.n_ref || npos < -1) { ++up; continue; }
    const int32_t next_up = up + 1;
    up -= 4;
    if (gb_seek(g.bz, g.in, cpv | (uint32_t)(up + 12))) return -1;
    if (gb_read(g.bz, g.in, g.buf, 4, &got)) return -1;
    const int32_t name_len = gbuf_i32(g, 0) & 0xff;
    const int32_t nul = up + 36 + name_len - 1;
    if (nul >= csize) { up = next_up; continue; }
    if (gb_seek(g.bz, g.in, cpv | (uint32_t)nul)) return -1;
    if (gb_read(g.bz, g.in, g.buf, 1, &got)) return -1;
    if (g.buf[0] != 0) { up = next_up; continue; }
    int32_t zero_min = 32 + name_len;
    if (gb_seek(g.bz, g.in, cpv | (uint32_t)(up + 16))) return -1;
    if (gb_read(g.bz, g.in, g.buf, 8, &got)) return -1;
    zero_min = (int32_t)((uint32_t)zero_min + (uint32_t)(gbuf_i32(g, 0) & 0xffff) * 4u);
    const int32_t ls = gbuf_i32(g, 4);
    const int32_t half = (int32_t)((uint32_t)ls + 1u) / 2;
    zero_min = (int32_t)((uint32_t)zero_min + (uint32_t)ls + (uint32_t)half);
    if (gb_seek(g.bz, g.in, cpv | (uint32_t)up)) return -1;
    if (gb_read(g.bz, g.in, g.buf, 4, &got)) return -1;
    if (gbuf_i32(g, 0) < zero_min) { up = next_up; continue; }
    return up;
  }
  return -1;
}

// Candidate blocks of each guess window: every offset of the window (the bytes
// BAMSplitGuesser's stream can reach, :118-126) that starts with the gzip magic 1f 8b 08 04.
// One workgroup per window; sorted by rank; count > GC_CAP marks the window uncached.
// bytes of guess g's window the state machine can reach: min((int)(end-beg), cap, available)
__device__ __forceinline__ int64_t g_window_total(int64_t b0, int64_t e0, int64_t avail, int32_t cap) {
  int32_t want = (int32_t)(e0 - b0);  // (int) cast as BAMSplitGuesser.java:118
  if (want > cap) want = cap;
  return (want > 0 && b0 >= 0) ? (avail < want ? avail : want) : 0;
}

__global__ __launch_bounds__(256) void k_guess_cands(const uint64_t* __restrict__ wptr,
                                                     const int64_t* __restrict__ wlen,
                                                     const int64_t* __restrict__ beg,
                                                     const int64_t* __restrict__ end,
                                                     uint32_t* __restrict__ cn,
                                                     uint64_t* __restrict__ cpos_slots) {
  __shared__ uint32_t s_n;
  __shared__ uint64_t s_p[GC_CAP];
  const uint32_t g = blockIdx.x;
  const int64_t b0 = beg[g];
  const int64_t total = g_window_total(b0, end[g], wlen[g], G_MAX_BYTES_READ);
  const uint8_t* w = (const uint8_t*)wptr[g];
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  for (int64_t p = threadIdx.x; p + 4 <= total; p += 256) {
    const uint8_t* q = w + p;
    if (q[0] == 0x1f && q[1] == 0x8b && q[2] == 8 && q[3] == 4) {
      const uint32_t k = atomicAdd(&s_n, 1u);
      if (k < GC_CAP) s_p[k] = (uint64_t)(b0 + p);
    }
  }
  __syncthreads();
  const uint32_t n = s_n;
  if (n > GC_CAP) {
    if (threadIdx.x == 0) cn[g] = n;
    return;
  }
  uint64_t v = 0;
  uint32_t r = 0;
  if (threadIdx.x < n) {
    v = s_p[threadIdx.x];
    for (uint32_t j = 0; j < n; ++j) r += s_p[j] < v ? 1u : 0u;
  }
  __syncthreads();
  if (threadIdx.x < n) cpos_slots[(uint64_t)g * GC_CAP + r] = v;
  if (threadIdx.x == 0) cn[g] = n;
}

__global__ void k_guess_clamp(const uint32_t* __restrict__ cn, uint32_t k, uint32_t* __restrict__ out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < k) out[g] = cn[g] <= GC_CAP ? cn[g] : 0u;
}

// Compact the per-window candidate slots and build their block records.  pad = 1 marks a
// block the cache inflates (whole block inside the window, 26 <= BSIZE+1, ISIZE <= 65536; the
// state machine cannot read a block that runs past the window: :94 of gb_read_block).
// BlockRec.coff is the block's device address (the batched inflate reads comp + coff with
// comp = nullptr); cpos keeps the absolute file offset the lookups search.
__global__ void k_guess_cand_blocks(const uint64_t* __restrict__ wptr, const int64_t* __restrict__ wlen,
                                    const int64_t* __restrict__ beg, const int64_t* __restrict__ end,
                                    uint32_t k,
                                    const uint32_t* __restrict__ cn, const uint64_t* __restrict__ cbase,
                                    const uint64_t* __restrict__ cpos_slots,
                                    uint64_t* __restrict__ cpos, BlockRec* __restrict__ cblk,
                                    uint32_t* __restrict__ cisz) {
  const uint32_t g = blockIdx.x;
  if (g >= k) return;
  const uint32_t n = cn[g] <= GC_CAP ? cn[g] : 0u;
  const uint64_t o = cbase[g];
  const int64_t b0 = beg[g];
  const int64_t total = g_window_total(b0, end[g], wlen[g], G_MAX_BYTES_READ);
  const uint8_t* w = (const uint8_t*)wptr[g];
  for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
    const uint64_t p = cpos_slots[(uint64_t)g * GC_CAP + j];
    const int64_t pr = (int64_t)p - b0;  // window-relative
    BlockRec r;
    r.coff = (uint64_t)(uintptr_t)(w + pr);
    r.clen = 0;
    r.isize = 0;
    r.crc = 0;
    r.pad = 0;
    if (pr + 18 <= total) {
      const uint32_t bl = (uint32_t)(w[pr + 16] | w[pr + 17] << 8) + 1u;
      if (bl >= 26 && pr + (int64_t)bl <= total) {
        const uint8_t* f = w + pr + bl - 8;
        const uint32_t crc = (uint32_t)f[0] | (uint32_t)f[1] << 8 | (uint32_t)f[2] << 16 | (uint32_t)f[3] << 24;
        const uint32_t isz = (uint32_t)f[4] | (uint32_t)f[5] << 8 | (uint32_t)f[6] << 16 | (uint32_t)f[7] << 24;
        if (isz <= 65536u) {
          r.clen = bl;
          r.isize = isz;
          r.crc = crc;
          r.pad = 1;
        }
      }
    }
    cpos[o + j] = p;
    cblk[o + j] = r;
    cisz[o + j] = r.isize;
  }
}

__device__ void crc_table_init(uint32_t* T) {
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? 0xedb88320u ^ (c >> 1) : c >> 1;
    T[i] = c;
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------------
// One WAVE per guess (k_guess_bam_wave): the reference state machine above still runs, in
// lockstep on every lane (uniform values, so each load is one request), but its two byte-by-byte
// searches are answered by the wave in parallel:
//   * guessNextBGZFPos' magic scan (:229-247): the window's magic positions in [0, firstEnd]
//     are listed once by 64 lanes; the scan's result from p is the first listed position q >= p
//     with q < firstEnd or q == p (the skip rule never steps over a magic, and the end test
//     only follows an advance).  Windows shorter than firstEnd + 4 (where a 4-byte read can be
//     short and leave stale bytes in `buf`) take the lane-serial path.
//   * guessNextBAMPos' candidate loop (:301-398): bam_pred() is the loop's test as a pure
//     function of the inflated block (every read lies inside it), evaluated for 64 offsets at
//     a time.  The serial g_next_bam is then run on the accepted offset (or the last one
//     tested) alone, which leaves the stream, the BlockCompressedInputStream and the 8-byte
//     buffer exactly as the full serial loop would.
// ------------------------------------------------------------------------------------------
constexpr uint32_t GW_MAG = 512;  // magic positions listed per window (more: lane-serial path)

__device__ __forceinline__ int32_t le32(const uint8_t* u, int32_t o) {
  return (int32_t)((uint32_t)u[o] | (uint32_t)u[o + 1] << 8 | (uint32_t)u[o + 2] << 16 |
                   (uint32_t)u[o + 3] << 24);
}
// guessNextBAMPos' test at candidate c (needs c + 39 < csize): refID/pos, mate refID/pos in
// [-1, n_ref] / >= -1, NUL at the end of the read name, block_size >= the fixed lengths
__device__ __forceinline__ bool bam_pred(const uint8_t* u, int32_t c, int32_t csize, int32_t n_ref) {
  const int32_t id = le32(u, c + 4), pos = le32(u, c + 8);
  if (id < -1 || id > n_ref || pos < -1) return false;
  const int32_t nid = le32(u, c + 24), npos = le32(u, c + 28);
  if (nid < -1 || nid > n_ref || npos < -1) return false;
  const int32_t name_len = u[c + 12];
  const int32_t nul = c + 36 + name_len - 1;
  if (nul >= csize || u[nul] != 0) return false;
  int32_t zero_min = 32 + name_len;
  zero_min = (int32_t)((uint32_t)zero_min + (uint32_t)(u[c + 16] | u[c + 17] << 8) * 4u);
  const int32_t ls = le32(u, c + 20);
  const int32_t half = (int32_t)((uint32_t)ls + 1u) / 2;
  zero_min = (int32_t)((uint32_t)zero_min + (uint32_t)ls + (uint32_t)half);
  return le32(u, c) >= zero_min;
}

// guessNextBGZFPos from p with the magic scan answered by the wave's list (see above)
__device__ bool g_next_bgzf_listed(Guesser& g, int32_t p, int32_t end, const int32_t* mag,
                                   uint32_t nmag, int32_t* opos, int32_t* osize) {
  for (;;) {
    if (!gs_seek(g.in, p)) return false;
    uint32_t lo = 0, hi = nmag;  // first listed position >= p
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (mag[mid] < p) lo = mid + 1;
      else hi = mid;
    }
    if (lo == nmag) return false;
    const int32_t q = mag[lo];
    if (q != p && q >= end) return false;
    p = q;
    gs_seek(g.in, p);
    gs_read(g.in, g.buf, 4);  // the read that matched: buf = the magic, pos = p + 4
    const int32_t p0 = p;
    p += 10;
    if (!gs_seek(g.in, p)) return false;
    gs_read(g.in, g.buf, 2);
    p += 2;
    const int32_t xlen = gbuf_u16(g, 0);
    const int32_t sub_end = p + xlen;
    while (p < sub_end) {
      gs_read(g.in, g.buf, 4);
      if (gbuf_i32(g, 0) != G_MAGIC_SUB) {
        p += 4 + gbuf_u16(g, 2);
        if (!gs_seek(g.in, p)) return false;
        continue;
      }
      gs_read(g.in, g.buf, 2);
      const int32_t bsize = gbuf_u16(g, 0);
      p += 6;
      while (p < sub_end) {
        if (!gs_seek(g.in, p)) return false;
        gs_read(g.in, g.buf, 4);
        p += 4 + gbuf_u16(g, 2);
      }
      if (p != sub_end) break;
      p += bsize - xlen - 19 + 4;
      if (!gs_seek(g.in, p)) return false;
      gs_read(g.in, g.buf, 4);
      *opos = p0;
      *osize = gbuf_i32(g, 0);
      return true;
    }
    p = p0 + 4;
  }
}

// guessNextBAMPos(cpv, up, csize) with the candidate loop evaluated by the wave
__device__ int32_t g_next_bam_wave(Guesser& g, uint64_t cpv, int32_t up, int32_t csize, uint32_t lane) {
  if (up + 39 >= csize) return -1;  // the serial loop would not read at all
  // the serial loop's first seek (re-reads the block if the BCIS moved on)
  if (gb_seek(g.bz, g.in, cpv | (uint32_t)(up + 4))) return -1;
  const uint8_t* u = g.bz.cur;
  const int32_t last = csize - 40;
  for (int32_t c0 = up; c0 <= last; c0 += 64) {
    const int32_t c = c0 + (int32_t)lane;
    const bool ok = c <= last && bam_pred(u, c, csize, g.n_ref);
    const uint64_t m = __ballot(ok);
    if (m) {
      const int32_t hit = c0 + (int32_t)(__ffsll((unsigned long long)m) - 1);
      return g_next_bam(g, cpv, hit, csize);  // == hit, with the serial loop's side effects
    }
  }
  return g_next_bam(g, cpv, last, csize);  // == -1; buf / cursor as after the last test
}

// Record-chain memo of one candidate block cp0.  A candidate's verdict (the codec loop of
// :171-192) is a pure function of where its chain starts: gb_seek(cp0|up) leaves the same
// stream state for every up, and the loop's (b, prev) are still (0, cp0) at every record start
// inside cp0.  So every record start x inside cp0 that a chain decoded leads to the same end
// (rc, b) and the same final stream state; a later candidate, or a later chain, that reaches x
// takes that end without re-decoding (decoded_any = true, since x decodes).  Near the window
// end, where every chain runs out of bytes, this turns the quadratic candidate walk of
// :159-208 linear.  An end whose block lives in the in-lane scratch is not memoised (the next
// candidate's seek overwrites the scratch).
constexpr int32_t GW_MEMO = 1024;  // record starts remembered per chain
struct ChainMemo {
  uint16_t* pos[2];  // LDS: ascending record starts of the remembered chain / the chain in flight
  int32_t n, cur;    // remembered count, cursor of the chain in flight
  int64_t s_fpos;    // stream state inside cp0 the remembered chain started from
  int32_t s_last_len, s_cur_len;
  const uint8_t* s_cur;
  int32_t rc, b;     // the end every remembered start leads to
  int64_t block_addr, fpos;
  int32_t last_len, cur_len, cur_off;
  const uint8_t* cur_p;
};

#ifdef HBAM_PROF
__device__ unsigned long long* g_gprof = nullptr;   // 8 u64 per guess (tools/prof_regions.py)
__device__ unsigned long long* g_gtrace = nullptr;  // guess g_gtrace_idx's candidates: [0] = count,
                                                    // then 2 u64 each (tools/diag_guess.py);
                                                    // its cache at [8193..]: 4 u64 per block
__device__ unsigned int g_gtrace_idx = 0;
#endif
// guessNextBAMRecordStart :109-212, one wave
#ifdef HBAM_PROF
#define GP_T(i)                                          \
  do {                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();    \
    gp[i] += t_ - gq;                                    \
    gq = t_;                                             \
  } while (0)
#define GP_C(i) (++gp[i])
#else
#define GP_T(i) \
  do {          \
  } while (0)
#define GP_C(i) (void)0
#endif
__device__ int64_t g_guess_wave(Guesser& g, const uint8_t* win, int64_t wavail, int64_t beg, int64_t end,
                                int32_t* err, int32_t* s_mag, uint32_t* s_nmag, uint16_t* s_memo,
                                uint32_t lane
#ifdef HBAM_PROF
                                , uint64_t* gp
#endif
                                ) {
#ifdef HBAM_PROF
  uint64_t gq = __builtin_amdgcn_s_memtime();
#endif
  *err = HBAM_OK;
  const int64_t total = g_window_total(beg, end, wavail, G_MAX_BYTES_READ);
  g.in.a = win;
  g.in.len = total;
  g.in.pos = 0;
  g.bz.wbase = beg >= 0 ? beg : 0;
  g.bz.block_addr = 0;
  g.bz.last_len = 0;
  g.bz.cur_len = -1;
  g.bz.cur_off = 0;
  int32_t first_end = (int32_t)(end - beg);
  if (first_end > 0xffff) first_end = 0xffff;
  // list the window's magic positions in [0, first_end] (in order)
  bool listed = first_end >= 0 && total >= (int64_t)first_end + 4;
  if (listed) {
    if (lane == 0) *s_nmag = 0;
    __syncthreads();
    uint32_t n = 0;
    for (int32_t p0 = 0; p0 <= first_end; p0 += 64) {
      const int32_t p = p0 + (int32_t)lane;
      const bool mm = p <= first_end && g.in.a[p] == 0x1f && g.in.a[p + 1] == 0x8b &&
                      g.in.a[p + 2] == 8 && g.in.a[p + 3] == 4;
      const uint64_t bm = __ballot(mm);
      if (mm) {
        const uint32_t k = n + lane_rank(bm);
        if (k < GW_MAG) s_mag[k] = p;
      }
      n += (uint32_t)__popcll(bm);
    }
    listed = n <= GW_MAG;
    if (lane == 0) *s_nmag = n;
    __syncthreads();
  }
  const uint32_t nmag = listed ? *s_nmag : 0u;
#ifdef HBAM_PROF
  gp[7] = listed ? nmag : 100000u;
#endif
  GP_T(0);  // magic listing
  ChainMemo mm;
  mm.pos[0] = s_memo;
  mm.pos[1] = s_memo + GW_MEMO;
  for (int32_t cp = 0;; ++cp) {
    int32_t ppos, psize;
    GP_C(4);
    const bool found = listed ? g_next_bgzf_listed(g, cp, first_end, s_mag, nmag, &ppos, &psize)
                              : g_next_bgzf(g, cp, first_end, &ppos, &psize);
    GP_T(1);
    if (!found) return end;
    const int32_t cp0 = cp = ppos;
    const uint64_t cpv = (uint64_t)(uint32_t)cp0 << 16;
    if (gb_seek(g.bz, g.in, cpv)) continue;  // catch (Throwable)
    GP_T(1);
    mm.n = 0;
    for (int32_t up = 0;; ++up) {
      GP_C(5);
      const int32_t up0 = up = g_next_bam_wave(g, cpv, up, psize, lane);
      GP_T(2);
      if (up0 < 0) break;
      if (gb_seek(g.bz, g.in, cpv | (uint32_t)up0)) { *err = HBAM_EIO; return end; }
      bool decoded_any = false;
      int b = 0;
      int32_t prev = cp0;
      int32_t rc = 0;
      int32_t nn = 0;  // starts of this chain inside cp0, into mm.pos[1]
      bool memo_hit = false;
      mm.cur = 0;
      // same cp0 stream state as the remembered chain (the first seek into cp0 may reuse a block
      // the previous candidate block's chain left behind, with the stream elsewhere)
      const int64_t s_fpos = g.in.pos;
      const int32_t s_last_len = g.bz.last_len, s_cur_len = g.bz.cur_len;
      const uint8_t* s_cur = g.bz.cur;
      const bool memo_ok = mm.n > 0 && mm.s_fpos == s_fpos && mm.s_last_len == s_last_len &&
                           mm.s_cur_len == s_cur_len && mm.s_cur == s_cur;
      while (b < 3) {
        if (b == 0 && memo_ok) {
          const int32_t x = g.bz.cur_off;
          while (mm.cur < mm.n && (int32_t)mm.pos[0][mm.cur] < x) ++mm.cur;
          if (mm.cur < mm.n && (int32_t)mm.pos[0][mm.cur] == x) {
            memo_hit = true;
            break;
          }
        }
        const int32_t x0 = g.bz.cur_off;
        rc = gc_decode(g.bz, g.in);
        GP_C(6);
        if (rc <= 0) break;
        if (b == 0 && nn < GW_MEMO) mm.pos[1][nn++] = (uint16_t)x0;
        decoded_any = true;
        const int32_t cp2 = (int32_t)(gb_tell(g.bz) >> 16);
        if (cp2 != prev) { prev = cp2; ++b; }
      }
      if (memo_hit) {  // this chain joins the remembered one: take its end
        rc = mm.rc;
        b = mm.b;
        decoded_any = true;
        g.bz.block_addr = mm.block_addr;
        g.bz.last_len = mm.last_len;
        g.bz.cur_len = mm.cur_len;
        g.bz.cur_off = mm.cur_off;
        g.bz.cur = mm.cur_p;
        g.in.pos = mm.fpos;
      } else if (nn > 0 && !(g.bz.cur == g.bz.scratch && g.bz.cur_len >= 0)) {
        uint16_t* t = mm.pos[0];  // remember this chain instead
        mm.pos[0] = mm.pos[1];
        mm.pos[1] = t;
        mm.n = nn;
        mm.s_fpos = s_fpos;
        mm.s_last_len = s_last_len;
        mm.s_cur_len = s_cur_len;
        mm.s_cur = s_cur;
        mm.rc = rc;
        mm.b = b;
        mm.block_addr = g.bz.block_addr;
        mm.last_len = g.bz.last_len;
        mm.cur_len = g.bz.cur_len;
        mm.cur_off = g.bz.cur_off;
        mm.cur_p = g.bz.cur;
        mm.fpos = g.in.pos;
      }
      GP_T(3);
#ifdef HBAM_PROF
      if (g_gtrace && blockIdx.x == g_gtrace_idx && lane == 0) {
        const unsigned long long k = g_gtrace[0];
        if (k < 4096) {
          g_gtrace[1 + 2 * k] = (unsigned long long)(uint32_t)cp0 << 32 | (uint32_t)up0;
          g_gtrace[2 + 2 * k] = (unsigned long long)(uint32_t)rc << 32 | (uint32_t)b << 8 |
                                (decoded_any ? 1u : 0u) | (memo_hit ? 2u : 0u);
          g_gtrace[0] = k + 1;
        }
      }
#endif
      if (rc < 0) {
        if (rc == HBAM_EFORMAT || rc == HBAM_ETRUNC || rc == HBAM_ERUNTIMEIO || rc == HBAM_EREFID)
          continue;
        if (rc == HBAM_EEOF) {
          if (!decoded_any && g.in.pos == g.in.len) continue;
        } else {
          *err = rc;
          return end;
        }
      } else if (b < 3) {
        if (!decoded_any) continue;
      }
      return (int64_t)((uint64_t)(beg + cp0) << 16 | (uint32_t)up0);
    }
  }
}

__global__ __launch_bounds__(64) void k_guess_bam_wave(const uint64_t* __restrict__ wptr,
                                                       const int64_t* __restrict__ wlen,
                                                       const int64_t* __restrict__ beg,
                                                       const int64_t* __restrict__ end, uint32_t k,
                                                       int32_t n_ref, uint8_t* __restrict__ scratch,
                                                       uint8_t* __restrict__ lens_scratch,
                                                       uint8_t* __restrict__ bufs,
                                                       int64_t* __restrict__ out,
                                                       int32_t* __restrict__ err,
                                                       const uint32_t* __restrict__ cn,
                                                       const uint64_t* __restrict__ cbase,
                                                       const uint64_t* __restrict__ cpos,
                                                       const BlockRec* __restrict__ cblk,
                                                       const uint64_t* __restrict__ cuoff,
                                                       const uint8_t* __restrict__ cubuf,
                                                       const int32_t* __restrict__ cst,
                                                       const uint32_t* __restrict__ ccrc) {
  __shared__ uint16_t s_ll[288];
  __shared__ uint8_t s_d[32];
  __shared__ uint32_t T[256];
  __shared__ int32_t s_mag[GW_MAG];
  __shared__ uint32_t s_nmag;
  __shared__ uint16_t s_memo[2 * GW_MEMO];
  crc_table_init(T);
  const uint32_t i = blockIdx.x, lane = threadIdx.x;
  if (i >= k) return;
  Guesser g;
  g.n_ref = n_ref;
  for (int j = 0; j < 8; ++j) g.buf[j] = bufs[8 * (uint64_t)i + j];
  g.bz.scratch = scratch + (uint64_t)i * 65536;
  g.bz.cur = g.bz.scratch;
  g.bz.cache.n = 0;
  if (cn && cn[i] <= GC_CAP) {
    const uint64_t o = cbase[i];
    g.bz.cache.n = cn[i];
    g.bz.cache.pos = cpos + o;
    g.bz.cache.blk = cblk + o;
    g.bz.cache.uoff = cuoff + o;
    g.bz.cache.ubuf = cubuf;
    g.bz.cache.st = cst + o;
    g.bz.cache.crc = ccrc + o;
  }
  g.bz.s_ll = s_ll;
  g.bz.s_d = s_d;
  g.bz.lens = lens_scratch + (uint64_t)i * LENS_SLOT;
  g.bz.crc_tab = T;
  g.bz.check_crc = 1;
  int32_t e;
#ifdef HBAM_PROF
  if (g_gtrace && i == g_gtrace_idx && lane == 0) {
    unsigned long long* q = g_gtrace + 8193;
    q[0] = g.bz.cache.n;
    for (uint32_t j = 0; j < g.bz.cache.n && j < 512; ++j) {
      q[1 + 4 * j] = g.bz.cache.pos[j];
      q[2 + 4 * j] = (unsigned long long)g.bz.cache.blk[j].clen << 32 | g.bz.cache.blk[j].isize;
      q[3 + 4 * j] = (unsigned long long)(uint32_t)g.bz.cache.st[j] << 32 | g.bz.cache.crc[j];
      q[4 + 4 * j] = (unsigned long long)g.bz.cache.blk[j].crc << 32 | g.bz.cache.blk[j].pad;
    }
  }
  uint64_t gp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const int64_t r = g_guess_wave(g, (const uint8_t*)wptr[i], wlen[i], beg[i], end[i], &e, s_mag, &s_nmag, s_memo, lane, gp);
  if (g_gprof && lane == 0) {
    gp[0] = __builtin_amdgcn_s_memtime() - t0;  // slot 0: whole guess (listing folded in below)
    for (int q = 0; q < 8; ++q) g_gprof[8 * (uint64_t)i + q] = gp[q];
  }
#else
  const int64_t r = g_guess_wave(g, (const uint8_t*)wptr[i], wlen[i], beg[i], end[i], &e, s_mag, &s_nmag, s_memo, lane);
#endif
  if (lane == 0) {
    out[i] = r;
    err[i] = e;
    for (int j = 0; j < 8; ++j) bufs[8 * (uint64_t)i + j] = g.buf[j];
  }
}

// BGZFSplitGuesser.guessNextBGZFBlockStart :51-92 (its own scan :95-148, IOExceptions escape)
constexpr int32_t G_BGZF_WINDOW = 2 * 0xffff - 1;  // BGZFSplitGuesser.java:62-63
__global__ __launch_bounds__(GUESS_WG) void k_guess_bgzf(const uint64_t* __restrict__ wptr,
                                                         const int64_t* __restrict__ wlen,
                                                         const int64_t* __restrict__ beg,
                                                         const int64_t* __restrict__ end, uint32_t k,
                                                         uint8_t* __restrict__ scratch,
                                                         uint8_t* __restrict__ lens_scratch,
                                                         int64_t* __restrict__ out,
                                                         int32_t* __restrict__ err) {
  __shared__ uint16_t s_ll[GUESS_WG * 288];
  __shared__ uint8_t s_d[GUESS_WG * 32];
  __shared__ uint32_t T[256];
  crc_table_init(T);
  const uint32_t i = blockIdx.x * GUESS_WG + threadIdx.x;
  if (i >= k) return;
  const int64_t b0 = beg[i], e0 = end[i];
  const int64_t total = g_window_total(b0, e0, wlen[i], G_BGZF_WINDOW);
  GStream in{(const uint8_t*)wptr[i], total, 0};
  GBcis bz;
  bz.block_addr = 0;
  bz.last_len = 0;
  bz.cur_len = -1;
  bz.cur_off = 0;
  bz.scratch = scratch + (uint64_t)i * 65536;
  bz.cur = bz.scratch;
  bz.wbase = b0 >= 0 ? b0 : 0;
  bz.cache.n = 0;
  bz.s_ll = s_ll + threadIdx.x * 288;
  bz.s_d = s_d + threadIdx.x * 32;
  bz.lens = lens_scratch + (uint64_t)i * LENS_SLOT;
  bz.crc_tab = T;
  bz.check_crc = 1;
  uint8_t buf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int32_t first_end = (int32_t)(e0 - b0);
  if (first_end > 0xffff) first_end = 0xffff;
  int64_t result = e0;
  int32_t e = HBAM_OK;
  auto i32 = [&](int o) {
    return (int32_t)((uint32_t)buf[o] | (uint32_t)buf[o + 1] << 8 | (uint32_t)buf[o + 2] << 16 |
                     (uint32_t)buf[o + 3] << 24);
  };
  for (int32_t pos = 0;;) {
    int32_t p = pos;
    bool found = false, notfound = false;
    for (;;) {
      for (;;) {
        if (!gs_seek(in, p)) { e = HBAM_EIO; goto done; }
        gs_read(in, buf, 4);
        const int32_t n = i32(0);
        if (n == G_MAGIC) break;
        if ((int32_t)((uint32_t)n >> 8) == 0x00088b1f) ++p;
        else if ((int32_t)((uint32_t)n >> 16) == 0x00008b1f) p += 2;
        else p += 3;
        if (p >= first_end) { notfound = true; break; }
      }
      if (notfound) break;
      const int32_t p0 = p;
      p += 10;
      if (!gs_seek(in, p)) { e = HBAM_EIO; goto done; }
      gs_read(in, buf, 2);
      p += 2;
      const int32_t xlen = (int32_t)(buf[0] | buf[1] << 8);
      const int32_t sub_end = p + xlen;
      while (p < sub_end) {
        gs_read(in, buf, 4);
        if (i32(0) != G_MAGIC_SUB) {
          p += 4 + (int32_t)(buf[2] | buf[3] << 8);
          if (!gs_seek(in, p)) { e = HBAM_EIO; goto done; }
          continue;
        }
        pos = p0;
        found = true;
        break;
      }
      if (found) break;
      p = p0 + 4;
    }
    if (notfound) { result = e0; break; }
    if (gb_seek(bz, in, (uint64_t)(uint32_t)pos << 16)) { ++pos; continue; }
    result = b0 + pos;
    break;
  }
done:
  out[i] = result;
  err[i] = e;
}

}  // namespace hbam
