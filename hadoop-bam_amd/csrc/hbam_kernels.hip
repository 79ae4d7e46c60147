// hbam_kernels.hip — MI355X (gfx950) kernels of the BAM read path.
//
// Stage map (SURVEY.md §2.1 build units -> reference hot loops):
//   K1 k_scan_chunks/k_gather_cands/k_verify_chain  BGZF framing   [htsjdk] BCIS.readBlock header
//                                                    parse; BGZFBlockIndexer.skipBlock :130-181
//   K2 k_inflate                                     [htsjdk] BlockGunzipper.unzipBlock (zlib)
//      k_crc32                                       CRC32 check (BCIS.setCheckCrcs)
//   K5 k_block_entry/k_block_walk/k_chain_fix/k_emit record boundaries: BAMRecordReader
//                                                    .nextKeyValue loop :172-188 -> decode()
//   K6/K7 k_decode_fixed / k_decode_pools            [htsjdk] BAMRecordCodec.decode + BAMRecord
//                                                    lazy getters; BAMRecordReader.getKey :66-106
//                                                    + MurmurHash3.murmurhash3 :32-102
//   K8 (in k_decode_fixed)                           split bound, BAMRecordReader.java:173
//
// Memory layout in HBM: comp = compressed file bytes (+64 B pad); ubuf = concatenation of
// the inflated blocks of the split (block b at uoff[b]); record starts rec_off (u64) into
// ubuf; struct-of-arrays columns; variable-length pools addressed by exclusive scans.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbam_internal.h"
#include "inflate_dev.h"
#include "inflate_tok.h"
#include "inflate_wave.h"
#include "resolve_dev.h"

namespace hbam {

// Byte-aligned scalar fields as one global load each: the device runs in unaligned access mode
// (as the LZ77 pass's 8-byte source loads rely on), so a 1-aligned u32 type compiles to a single
// global_load_dword instead of four byte loads and three shifts.
typedef uint32_t u32_a1 __attribute__((aligned(1)));
typedef uint16_t u16_a1 __attribute__((aligned(1)));
static __device__ __forceinline__ uint32_t ld_u32_unaligned(const uint8_t* p) { return *(const u32_a1*)p; }
static __device__ __forceinline__ uint16_t ld_u16_unaligned(const uint8_t* p) { return *(const u16_a1*)p; }

// ------------------------------------------------------------------------------------
// K1: candidate BGZF block starts.  htsjdk accepts a block when bytes 0..3 = 1f 8b 08 04
// and XLEN (u16 @10) == 6 (BlockGunzipper; SI1/SI2/SLEN are skipped unchecked); the block
// length is BSIZE (u16 @16) + 1.  One workgroup scans a SCAN_CHUNK-byte chunk; candidates
// are collected in LDS, sorted, and written to a per-chunk slot (cap SCAN_CAP).
// ------------------------------------------------------------------------------------
// Candidate test of the 16 positions [p0, p0 + 16): bit k set when p0 + k can start a block
// (the two-pass fallback; k_scan_chunks keeps its inline form: written with this helper it ran
// 1.59 -> 1.85 ms at 5 GB, profiles/r03/ab/pools_ilp_and_scan_5g.txt).
__device__ __forceinline__ uint32_t scan_mask16(const uint8_t* __restrict__ comp, uint64_t p0, uint64_t end) {
  // (two 16-byte loads instead of the dword loads: 3.07 -> 3.34 ms per 10 GB, not kept)
  uint32_t w[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) w[i] = ld_u32_unaligned(comp + p0 + 4 * i);
  uint32_t mask = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint64_t p = p0 + k;
    // bytes p..p+3 and p+10..p+11
    const int q = k >> 2, r = k & 3;
    const uint64_t lo = (uint64_t)w[q] | (uint64_t)w[q + 1] << 32;
    const uint32_t m = (uint32_t)(lo >> (8 * r));
    const uint64_t lo2 = (uint64_t)w[(k + 8) >> 2] | (uint64_t)w[((k + 8) >> 2) + 1] << 32;
    const uint32_t x = (uint32_t)(lo2 >> (8 * ((k + 8) & 3)));  // bytes p+8..p+11
    if (p + 18 <= end && m == 0x04088b1fu && (x >> 16) == 6u) mask |= 1u << k;
  }
  return mask;
}

__global__ __launch_bounds__(256) void k_scan_chunks(const uint8_t* __restrict__ comp,
                                                     uint64_t begin, uint64_t end,
                                                     uint32_t* __restrict__ chunk_cnt,
                                                     uint64_t* __restrict__ chunk_pos,
                                                     uint32_t* __restrict__ overflow) {
  __shared__ uint32_t s_cnt;
  __shared__ uint64_t s_pos[SCAN_CAP];
  const uint64_t chunk = blockIdx.x;
  const uint64_t c0 = begin + chunk * SCAN_CHUNK;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  // each thread tests 16 consecutive positions per step using a 32-byte window
  // (requesting the next step's window before testing this one: 1.56 -> 1.71 ms at 5 GB,
  // profiles/r03/ab/scan_prefetch_5g.txt; not kept)
// positions per thread per step: 16 -> 32 keeps twice the bytes in flight, 1.55 -> 1.40 ms at 5 GB
// (profiles/r04/ab/scan_32_positions_5g.txt)
constexpr int SCAN_POS = 32;
  constexpr int SP = SCAN_POS;
  for (uint32_t step = 0; step < SCAN_CHUNK / (256 * SP); ++step) {
    const uint64_t p0 = c0 + ((uint64_t)step * 256 + threadIdx.x) * SP;
    if (p0 >= end) break;
    // positions p0..p0+SP-1 need bytes up to p0 + SP + 11
    uint32_t w[SP / 4 + 3];
    // SP bytes per lane as 16-byte loads (a wave reads 2 KiB with no overlap), the 12 bytes after
    // them from the next lane by DPP wave_shl:1 (lane 63: one extra load of its own); against
    // SP/4 + 3 byte-aligned dword loads per lane (the last three overlapping the next lane's):
    // 1.346 -> 1.241 ms at 5 GB (profiles/r05/ab/scan_dpp_neighbour_5g.txt)
    static_assert(SP % 16 == 0, "scan: whole 16-byte loads per lane");
#pragma unroll
    for (int i = 0; i < SP / 16; ++i) {
      const u32x4_t q = *(const __attribute__((address_space(1))) u32x4_t*)(comp + p0 + 16 * i);
      w[4 * i] = q[0]; w[4 * i + 1] = q[1]; w[4 * i + 2] = q[2]; w[4 * i + 3] = q[3];
    }
    uint32_t x0 = 0, x1 = 0, x2 = 0;
    if ((threadIdx.x & 63u) == 63u) {
      x0 = ld_u32_unaligned(comp + p0 + SP);
      x1 = ld_u32_unaligned(comp + p0 + SP + 4);
      x2 = ld_u32_unaligned(comp + p0 + SP + 8);
    }
    // (a lane whose right neighbour has left the loop only needs neighbour bytes for positions
    // past `end`, which are not tested)
    w[SP / 4] = (uint32_t)__builtin_amdgcn_update_dpp((int)x0, (int)w[0], 0x130, 0xf, 0xf, false);
    w[SP / 4 + 1] = (uint32_t)__builtin_amdgcn_update_dpp((int)x1, (int)w[1], 0x130, 0xf, 0xf, false);
    w[SP / 4 + 2] = (uint32_t)__builtin_amdgcn_update_dpp((int)x2, (int)w[2], 0x130, 0xf, 0xf, false);
#pragma unroll
    for (int k = 0; k < SP; ++k) {
      const uint64_t p = p0 + k;
      if (p + 18 > end) break;
      // bytes p..p+3 and p+10..p+11
      const int q = k >> 2, r = k & 3;
      const uint64_t lo = (uint64_t)w[q] | (uint64_t)w[q + 1] << 32;
      const uint32_t m = (uint32_t)(lo >> (8 * r));
      const uint64_t lo2 = (uint64_t)w[(k + 8) >> 2] | (uint64_t)w[((k + 8) >> 2) + 1] << 32;
      const uint32_t x = (uint32_t)(lo2 >> (8 * ((k + 8) & 3)));  // bytes p+8..p+11
      if (m == 0x04088b1fu && (x >> 16) == 6u) {
        const uint32_t i = atomicAdd(&s_cnt, 1u);
        if (i < SCAN_CAP) s_pos[i] = p;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t n = s_cnt;
    if (n > SCAN_CAP) {
      atomicOr(overflow, 1u);
      n = SCAN_CAP;
    }
    // insertion sort (n is tiny: ~2-3 true blocks per 64 KiB)
    for (uint32_t i = 1; i < n; ++i) {
      const uint64_t v = s_pos[i];
      uint32_t j = i;
      while (j > 0 && s_pos[j - 1] > v) { s_pos[j] = s_pos[j - 1]; --j; }
      s_pos[j] = v;
    }
    chunk_cnt[chunk] = n;
    for (uint32_t i = 0; i < n; ++i) chunk_pos[chunk * SCAN_CAP + i] = s_pos[i];
  }
}

// Exact two-pass form of the candidate scan, for files whose blocks are so small (or whose
// data holds so many magic patterns) that a chunk has more than SCAN_CAP candidates: pass 1
// counts each chunk's candidates, pass 2 writes them at the chunk's exclusive-scan offset in
// position order (a workgroup scan of the per-thread counts at every step), straight into
// the candidate list.
__global__ __launch_bounds__(256) void k_scan_count(const uint8_t* __restrict__ comp, uint64_t begin,
                                                    uint64_t end, uint32_t* __restrict__ chunk_cnt) {
  __shared__ uint32_t s_cnt;
  const uint64_t c0 = begin + (uint64_t)blockIdx.x * SCAN_CHUNK;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  uint32_t n = 0;
  for (uint32_t step = 0; step < SCAN_CHUNK / (256 * 16); ++step) {
    const uint64_t p0 = c0 + ((uint64_t)step * 256 + threadIdx.x) * 16;
    if (p0 >= end) break;
    n += __popc(scan_mask16(comp, p0, end));
  }
  atomicAdd(&s_cnt, n);
  __syncthreads();
  if (threadIdx.x == 0) chunk_cnt[blockIdx.x] = s_cnt;
}
__global__ __launch_bounds__(256) void k_scan_write(const uint8_t* __restrict__ comp, uint64_t begin,
                                                    uint64_t end, const uint64_t* __restrict__ chunk_base,
                                                    uint64_t* __restrict__ cand) {
  __shared__ uint32_t s_wsum[4];
  const uint64_t c0 = begin + (uint64_t)blockIdx.x * SCAN_CHUNK;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint64_t run = chunk_base[blockIdx.x];
  for (uint32_t step = 0; step < SCAN_CHUNK / (256 * 16); ++step) {
    const uint64_t p0 = c0 + ((uint64_t)step * 256 + threadIdx.x) * 16;
    uint32_t mask = p0 < end ? scan_mask16(comp, p0, end) : 0u;
    const uint32_t cnt = __popc(mask);
    uint32_t incl = cnt;  // inclusive scan within the wave
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t t = __shfl_up(incl, off);
      if ((int)lane >= off) incl += t;
    }
    if (lane == 63) s_wsum[wv] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      before += j < wv ? s_wsum[j] : 0u;
      total += s_wsum[j];
    }
    uint64_t o = run + before + incl - cnt;
    while (mask) {
      const uint32_t k = __ffs(mask) - 1u;
      mask &= mask - 1u;
      cand[o++] = p0 + k;
    }
    run += total;
    __syncthreads();
  }
}

__global__ void k_gather_cands(const uint32_t* __restrict__ chunk_cnt,
                               const uint64_t* __restrict__ chunk_base,
                               const uint64_t* __restrict__ chunk_pos, uint64_t nchunks,
                               uint64_t* __restrict__ cand) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  const uint32_t n = chunk_cnt[c];
  const uint64_t b = chunk_base[c];
  for (uint32_t i = 0; i < n; ++i) cand[b + i] = chunk_pos[c * SCAN_CAP + i];
}

// Chain check: cand[0] must be the chain start; every candidate's successor
// (pos + BSIZE + 1) must be the next candidate (or the data end for the last).  Fills the
// block table on the way.
__global__ void k_verify_chain(const uint8_t* __restrict__ comp, const uint64_t* __restrict__ cand,
                               uint64_t n, uint64_t data_end, BlockRec* __restrict__ blk,
                               uint32_t* __restrict__ bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t p = cand[i];
  const uint32_t bl = (uint32_t)ld_u16_unaligned(comp + p + 16) + 1u;
  const uint64_t nx = p + bl;
  bool ok = (i + 1 < n) ? (nx == cand[i + 1]) : (nx <= data_end);
  BlockRec r;
  r.coff = p;
  r.clen = bl;
  if (nx <= data_end && bl >= 18) {
    r.crc = ld_u32_unaligned(comp + p + bl - 8);
    r.isize = ld_u32_unaligned(comp + p + bl - 4);
  } else {
    r.crc = 0;
    r.isize = 0;
    ok = false;
  }
  blk[i] = r;
  if (!ok) atomicAdd(bad, 1u);
}

// ------------------------------------------------------------------------------------
// K2: inflate = two kernels.
//  k_inflate_wave (phase 1, calls of up to WAVE_MAX_BLOCKS blocks): one wave per BGZF
//    block, same output; see inflate_wave.h.  Blocks it does not take go to k_inflate_tokens.
//  k_inflate_tokens (phase 1): one lane per BGZF block (SIMT across blocks); Huffman
//    decode with wave-uniform input epochs; literals land in ubuf, each match leaves a
//    3-byte descriptor in its hole and a bit in the block's match-start bitmap (TSink,
//    inflate_tok.h).  LDS: per lane 288 + 32 u8 symbol slots.
//  k_resolve_units (phase 2, LZ77): one wave per block walks it in 1 KiB stretches staged in
//    LDS; every match is cut into <= 16-byte units, copied all at once when their source is
//    final, in dataflow rounds otherwise (resolve_units.h).
// ------------------------------------------------------------------------------------
#ifdef HBAM_PROF
// Profiling build only (libhbam_prof.so, tools/profile_inflate.py --prof): per-block cycle
// counters, 16 u64 per block.
__device__ unsigned long long* g_prof = nullptr;
#define PROF_CLK() __builtin_amdgcn_s_memtime()
#define PROF_RT() __builtin_amdgcn_s_memrealtime()
#endif
#if defined(HBAM_PROF) || !defined(HBAM_SPLIT_TOK)
}  // namespace hbam
#include "hbam_inflate_tokens.hip"  // the Huffman lane pass in this translation unit
namespace hbam {
#else
// The Huffman lane pass is its own translation unit (hbam_inflate_tokens.hip), compiled with the
// max-ILP machine scheduler; see there.
__global__ void k_inflate_tokens(const uint8_t* __restrict__ comp, const BlockRec* __restrict__ blk,
                                 const uint64_t* __restrict__ uoff, uint32_t nblk, uint8_t* __restrict__ ubuf,
                                 uint8_t* __restrict__ lens_scratch, uint32_t* __restrict__ bitmap,
                                 uint32_t* __restrict__ tails, uint8_t* __restrict__ edges,
                                 int32_t* __restrict__ status, const uint32_t* __restrict__ list,
                                 const uint32_t* __restrict__ nlist);
#endif

// Huffman pass, one wave (= one workgroup) per BGZF block; see inflate_wave.h.  Blocks it does
// not take are appended to list for k_inflate_tokens.
__global__ __launch_bounds__(64, WV_WAVES) void k_inflate_wave(const uint8_t* __restrict__ comp,
                                                                   const BlockRec* __restrict__ blk,
                                                                   const uint64_t* __restrict__ uoff,
                                                                   uint32_t nblk, uint8_t* __restrict__ ubuf,
                                                                   uint32_t* __restrict__ bitmap,
                                                                   uint32_t* __restrict__ tails,
                                                                   uint8_t* __restrict__ edges,
                                                                   int32_t* __restrict__ status,
                                                                   uint32_t* __restrict__ list,
                                                                   uint32_t* __restrict__ nlist) {
  __shared__ WvLds S;
  const uint32_t b = blockIdx.x;
  if (b >= nblk) return;
  const BlockRec r = blk[b];
  bool ok = false;
  if (r.isize >= 64u && r.isize <= 65536u && r.clen >= 26u + 8u) {
    ok = inflate_wave_block(S, comp + r.coff + 18, r.clen - 26u, r.isize, ubuf, uoff[b],
                            bitmap + (uint64_t)b * BITMAP_WORDS, edges + 32 * (uint64_t)b);
  }
  if (threadIdx.x == 0) {
    if (ok) {
      tails[2 * (uint64_t)b] = 0;
      status[b] = INF_OK;
    } else {
      list[atomicAdd(nlist, 1u)] = b;
    }
  }
}

// The partial first / last chunks of each block (TSink edge slots) -> this block's bytes of
// them in ubuf.  One thread per (block, slot); neighbours write disjoint bytes of a shared
// chunk.  Runs between the Huffman pass and k_resolve.
__global__ void k_edge_merge(const BlockRec* __restrict__ blk, const uint64_t* __restrict__ uoff,
                             uint32_t nblk, uint8_t* __restrict__ ubuf, const uint8_t* __restrict__ edges) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t b = (uint32_t)(i >> 1), slot = (uint32_t)(i & 1);
  if (b >= nblk) return;
  const uint32_t isize = blk[b].isize;
  if (isize == 0 || isize > 65536u || blk[b].clen < 26u) return;  // no Huffman pass ran
  const uint64_t start = uoff[b];
  const uint32_t soff = (uint32_t)(start & 15u), iend = soff + isize;
  uint8_t* base = ubuf + (start & ~15ull);
  const uint8_t* src = edges + 32 * (uint64_t)b + 16u * slot;
  uint32_t lo, hi;
  if (slot == 0) {
    if (soff == 0) return;
    lo = soff;
    hi = iend < 16u ? iend : 16u;
  } else {
    const uint32_t cl = (iend - 1u) >> 4;
    if ((iend & 15u) == 0 || (cl == 0 && soff != 0)) return;
    lo = cl << 4;
    hi = iend;
  }
  for (uint32_t r = lo; r < hi; ++r) base[r] = src[r & 15u];
}

// one 16-byte column of a resolved stretch -> ubuf (bytewise where it overlaps a neighbour block)
__device__ __forceinline__ void rs_write_back(uint8_t* __restrict__ ubuf, uint64_t a, uint64_t base,
                                              uint64_t aend, const uint4 v) {
  if (a >= base && a + 16 <= aend) {
    *(uint4*)(ubuf + a) = v;
  } else if (a + 16 > base && a < aend) {
    for (uint32_t t = 0; t < 16; ++t) {
      const uint32_t wv = t < 4 ? v.x : t < 8 ? v.y : t < 12 ? v.z : v.w;
      if (a + t >= base && a + t < aend) ubuf[a + t] = (uint8_t)(wv >> (8 * (t & 3)));
    }
  }
}
// LZ77 resolution of one block (phase 2 of the batched inflate): k_resolve_units
#include "resolve_units.h"

// CRC-32 (IEEE, reflected 0xEDB88320) of each inflated block, slice-by-4 tables in LDS.
__global__ __launch_bounds__(256) void k_crc32(const BlockRec* __restrict__ blk,
                                               const uint64_t* __restrict__ uoff, uint32_t nblk,
                                               const uint8_t* __restrict__ ubuf,
                                               uint32_t* __restrict__ crc_out) {
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
  const uint8_t* p = ubuf + uoff[b];
  uint32_t n = blk[b].isize;
  uint32_t c = 0xffffffffu;
  while (n && ((uintptr_t)p & 3u)) { c = T[0][(c ^ *p++) & 0xff] ^ (c >> 8); --n; }
  const uint32_t* w = (const uint32_t*)p;
  for (; n >= 4; n -= 4) {
    c ^= *w++;
    c = T[3][c & 0xff] ^ T[2][(c >> 8) & 0xff] ^ T[1][(c >> 16) & 0xff] ^ T[0][c >> 24];
  }
  p = (const uint8_t*)w;
  while (n--) c = T[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  crc_out[b] = ~c;
}

// ------------------------------------------------------------------------------------
// K5: record boundaries over the inflated stream.  Chain: r_{k+1} = r_k + 4 + block_size_k.
// Per block: find an entry candidate (first offset passing a strict record predicate
// plus a short chain check), walk to the block end, then stitch: entry[b] must equal
// exit[b-1]; mismatches are re-walked in order by k_chain_fix.
// ------------------------------------------------------------------------------------
static __device__ __forceinline__ bool rec_plausible(const uint8_t* __restrict__ u, uint64_t x,
                                                     uint64_t hard_end, int32_t n_ref) {
  if (x + 36 > hard_end) return false;
  const uint8_t* p = u + x;
  const int32_t bs = (int32_t)ld_u32_unaligned(p);
  const int32_t id = (int32_t)ld_u32_unaligned(p + 4);
  const int32_t pos = (int32_t)ld_u32_unaligned(p + 8);
  const uint32_t L = p[12];
  const uint32_t ncig = ld_u16_unaligned(p + 16);
  const int32_t lseq = (int32_t)ld_u32_unaligned(p + 20);
  const int32_t nid = (int32_t)ld_u32_unaligned(p + 24);
  const int32_t npos = (int32_t)ld_u32_unaligned(p + 28);
  if (bs < 32 || id < -1 || id >= n_ref || nid < -1 || nid >= n_ref || pos < -1 || npos < -1)
    return false;
  if (L == 0 || lseq < 0) return false;
  const int64_t need = 32 + (int64_t)L + 4 * (int64_t)ncig + (int64_t)lseq + ((int64_t)lseq + 1) / 2;
  if ((int64_t)bs < need) return false;
  if (x + 36 + L > hard_end) return false;
  return p[36 + L - 1] == 0;
}

// The chain walk is generic over the record format: Fmt::plausible(u, x, hard_end) is the
// per-block entry predicate, Fmt::next(u, r, hard_end) the chain step from a record start
// (CHAIN_STOP where the record cannot be framed: the decode reports it).
struct BamFmt {  // BAMRecordCodec framing: r + 4 + block_size, block_size >= 32
  int32_t n_ref;
  __device__ __forceinline__ bool plausible(const uint8_t* __restrict__ u, uint64_t x, uint64_t hard_end) const {
    return rec_plausible(u, x, hard_end, n_ref);
  }
  __device__ __forceinline__ uint64_t next(const uint8_t* __restrict__ u, uint64_t r, uint64_t hard_end) const {
    if (r + 4 > hard_end) return CHAIN_STOP;
    const int32_t bs = (int32_t)ld_u32_unaligned(u + r);
    if (bs < 32) return CHAIN_STOP;
    return r + 4 + (uint64_t)(uint32_t)bs;
  }
};

template <typename Fmt>
__global__ __launch_bounds__(64) void k_block_entry(const uint8_t* __restrict__ u,
                                                    const uint64_t* __restrict__ uoff, uint32_t nblk,
                                                    uint64_t hard_end, Fmt fmt,
                                                    uint64_t* __restrict__ entry) {
  const uint32_t b = blockIdx.x + 1;  // block 0's entry is the split start
  if (b >= nblk) return;
  const uint64_t b0 = uoff[b], b1 = uoff[b + 1];
  const uint32_t lane = threadIdx.x;
  uint64_t found = NO_ENTRY;
  for (uint64_t x0 = b0; x0 < b1 && found == NO_ENTRY; x0 += 64) {
    const uint64_t x = x0 + lane;
    const bool c = (x < b1) && fmt.plausible(u, x, hard_end);
    uint64_t mask = __ballot(c);
    while (mask) {
      const int l = __ffsll((unsigned long long)mask) - 1;
      mask &= mask - 1;
      const uint64_t xc = x0 + (uint64_t)l;
      // chain check: up to 3 further hops must be plausible or end exactly at hard_end
      bool ok = true;
      if (lane == 0) {
        uint64_t r = xc;
        for (int h = 0; h < 3 && ok; ++h) {
          r = fmt.next(u, r, hard_end);
          if (r == hard_end) break;
          ok = r != CHAIN_STOP && fmt.plausible(u, r, hard_end);
        }
      }
      ok = __shfl(ok, 0);
      if (ok) { found = xc; break; }
    }
  }
  if (lane == 0) entry[b] = found;
}

// Walk block b from entry[b]: record starts in [uoff[b], uoff[b+1]) are stored as u16
// offsets (cap WALK_CAP per block); exit[b] = first chain position >= uoff[b+1], or
// CHAIN_STOP when a record cannot be framed (the chain ends there).
template <typename Fmt>
static __device__ void walk_one(const uint8_t* __restrict__ u, const uint64_t* __restrict__ uoff,
                                uint32_t b, uint64_t r, uint64_t hard_end, const Fmt& fmt,
                                uint16_t* __restrict__ rel, uint32_t* __restrict__ count,
                                uint64_t* __restrict__ exitp) {
  const uint64_t b0 = uoff[b], b1 = uoff[b + 1];
  uint32_t n = 0;
  if (r == NO_ENTRY) {
    count[b] = 0;
    exitp[b] = NO_ENTRY;
    return;
  }
  if (r == CHAIN_STOP) {
    count[b] = 0;
    exitp[b] = CHAIN_STOP;
    return;
  }
  // The offsets go out eight at a time as one 16-byte store (WALK_CAP and the block's slot are
  // multiples of 8 entries): a 2-byte store per record from a lane per block reached L2 as a
  // partial line each time (WRITE_SIZE 2.41 GB for 0.15 GB of offsets at config #2).
  static_assert(WALK_CAP % 8u == 0u, "walk: 16-byte groups of offsets");
  uint16_t* const rb = rel + (uint64_t)b * WALK_CAP;
  uint64_t lo = 0, hi = 0;  // the last <= 8 offsets, oldest in the low half-word of lo
  while (r < b1) {
    lo = (lo >> 16) | (hi << 48);
    hi = (hi >> 16) | (uint64_t)(uint16_t)(r - b0) << 48;
    ++n;
    if ((n & 7u) == 0u && n <= WALK_CAP)
      *(uint4*)(rb + n - 8u) = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
    r = fmt.next(u, r, hard_end);
    if (r == CHAIN_STOP) break;
  }
  for (uint32_t k = n & 7u, i = 0; i < k; ++i) {  // the last n % 8 offsets: the top k slots
    const uint32_t idx = n - k + i, slot = 8u - k + i;
    if (idx < WALK_CAP) rb[idx] = (uint16_t)(slot < 4u ? lo >> (16u * slot) : hi >> (16u * (slot - 4u)));
  }
  count[b] = n;
  exitp[b] = r;
}

template <typename Fmt>
__global__ void k_block_walk(const uint8_t* __restrict__ u, const uint64_t* __restrict__ uoff,
                             uint32_t nblk, uint64_t r0, uint64_t hard_end, Fmt fmt,
                             const uint64_t* __restrict__ entry, uint16_t* __restrict__ rel,
                             uint32_t* __restrict__ count, uint64_t* __restrict__ exitp) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  const uint64_t r = (b == 0) ? r0 : entry[b];
  walk_one(u, uoff, b, r, hard_end, fmt, rel, count, exitp);
}

// mismatch list: blocks whose entry != predecessor's exit (mark: 1 per listed block, optional)
__global__ void k_stitch_check(const uint64_t* __restrict__ entry, const uint64_t* __restrict__ exitp,
                               uint32_t nblk, uint32_t* __restrict__ nbad,
                               uint32_t* __restrict__ bad_list, uint32_t cap, uint8_t* __restrict__ mark) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (b >= nblk) return;
  const bool bad = entry[b] != exitp[b - 1];
  if (mark) mark[b] = bad ? 1 : 0;
  if (bad) {
    const uint32_t i = atomicAdd(nbad, 1u);
    if (i < cap) bad_list[i] = b;
  }
}

// Parallel repair: one lane per run of mismatched blocks.  A listed block whose predecessor is
// not listed heads a run; its lane re-walks it from the predecessor's exit and carries on while
// the next block is still inconsistent, stopping before the next run head (owned by another
// lane), so no two lanes write one block.  A head whose predecessor another lane re-walked may
// start from a stale exit: the stitch check after this pass catches that, and k_chain_fix
// finishes in order.
template <typename Fmt>
__global__ void k_chain_fix_par(const uint8_t* __restrict__ u, const uint64_t* __restrict__ uoff,
                                uint32_t nblk, uint64_t hard_end, Fmt fmt, uint64_t* __restrict__ entry,
                                uint16_t* __restrict__ rel, uint32_t* __restrict__ count,
                                uint64_t* __restrict__ exitp, const uint32_t* __restrict__ bad_list,
                                uint32_t nbad, const uint8_t* __restrict__ mark) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nbad) return;
  uint32_t b = bad_list[i];
  if (mark[b - 1]) return;  // not a run head
  for (;;) {
    const uint64_t e = exitp[b - 1];
    entry[b] = e;
    walk_one(u, uoff, b, e, hard_end, fmt, rel, count, exitp);
    ++b;
    if (b >= nblk || (mark[b] && !mark[b - 1])) break;  // the end, or the next run's head
    if (entry[b] == exitp[b - 1]) break;                 // consistent again
  }
}

// Sequential repair (one lane): process mismatched blocks in order, re-walking from the
// predecessor's exit and propagating until consistent again.
template <typename Fmt>
__global__ void k_chain_fix(const uint8_t* __restrict__ u, const uint64_t* __restrict__ uoff,
                            uint32_t nblk, uint64_t hard_end, Fmt fmt, uint64_t* __restrict__ entry,
                            uint16_t* __restrict__ rel, uint32_t* __restrict__ count,
                            uint64_t* __restrict__ exitp, const uint32_t* __restrict__ bad_list,
                            uint32_t nbad) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t done_upto = 0;  // blocks < done_upto are consistent
  for (uint32_t i = 0; i < nbad; ++i) {
    uint32_t b = bad_list[i];
    if (b < done_upto) continue;
    while (b < nblk && entry[b] != exitp[b - 1]) {
      const uint64_t e = exitp[b - 1];
      entry[b] = e;
      walk_one(u, uoff, b, e, hard_end, fmt, rel, count, exitp);
      ++b;
    }
    done_upto = b;
  }
}

// voffsets are FILE virtual offsets: block coffs are relative to the window, which starts at
// file offset comp_base
__global__ void k_emit_offsets(const uint64_t* __restrict__ uoff, const BlockRec* __restrict__ blk,
                               uint32_t nblk, const uint16_t* __restrict__ rel,
                               const uint32_t* __restrict__ count, const uint64_t* __restrict__ base,
                               uint64_t comp_base, uint64_t* __restrict__ rec_off,
                               uint64_t* __restrict__ voffset) {
  const uint32_t b = blockIdx.x;
  if (b >= nblk) return;
  const uint32_t n = count[b] < WALK_CAP ? count[b] : WALK_CAP;
  const uint64_t o = base[b];
  const uint64_t u0 = uoff[b];
  const uint64_t cv = (blk[b].coff + comp_base) << 16;
  for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
    const uint32_t r = rel[(uint64_t)b * WALK_CAP + k];
    rec_off[o + k] = u0 + r;
    voffset[o + k] = cv | r;
  }
}

// ------------------------------------------------------------------------------------
// K6/K7/K8: fixed-field decode, per-record status, coordinate key, pool lengths.
// ------------------------------------------------------------------------------------
static __device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return x << r | x >> (64 - r); }
static __device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}
static __device__ __forceinline__ uint64_t ld_u64_unaligned(const uint8_t* p) {
  return (uint64_t)ld_u32_unaligned(p) | (uint64_t)ld_u32_unaligned(p + 4) << 32;
}
// MurmurHash3.murmurhash3(byte[], seed=0) incl. the h2 quirk of MurmurHash3.java:59
// The 16-byte blocks are loaded MH_BATCH at a time, all loads of a batch in flight together,
// and the tail as two 8-byte loads (masked): an unmapped read's hash (the whole variable part,
// ~19 blocks) used to wait for one dependent load pair per block plus one per tail byte, and
// with ~1 % unmapped reads about half of the waves carried one such lane.
constexpr int32_t MH_BATCH = 8;  // 16-byte blocks of a murmur hash loaded together
static __device__ uint64_t murmur3_java(const uint8_t* __restrict__ key, int32_t len) {
  const int32_t nblocks = len / 16;
  uint64_t h1 = 0, h2 = 0;
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  for (int32_t i0 = 0; i0 < nblocks; i0 += MH_BATCH) {
    uint64_t kk[2 * MH_BATCH];
#pragma unroll
    for (int32_t j = 0; j < MH_BATCH; ++j) {
      const uint8_t* q = key + 16 * (i0 + j < nblocks ? i0 + j : i0);  // past the last block: re-read one
      kk[2 * j] = ld_u64_unaligned(q);
      kk[2 * j + 1] = ld_u64_unaligned(q + 8);
    }
#pragma unroll
    for (int32_t j = 0; j < MH_BATCH; ++j) {
      if (i0 + j < nblocks) {
        uint64_t k1 = kk[2 * j], k2 = kk[2 * j + 1];
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = h2 << 31 | h1 >> 33;
        h2 += h1; h2 = h2 * 5 + 0x38495ab5;
      }
    }
  }
  // tail: t < 16 bytes as little-endian words (over-reads stay inside ubuf + slack)
  const uint8_t* tail = key + 16 * nblocks;
  const int32_t t = len & 15;
  const uint64_t w0 = ld_u64_unaligned(tail), w1 = ld_u64_unaligned(tail + 8);
  const uint64_t k1 = t >= 8 ? w0 : (t > 0 ? w0 & ((1ull << (8 * t)) - 1ull) : 0ull);
  const uint64_t k2 = t > 8 ? w1 & (t == 16 ? ~0ull : ((1ull << (8 * (t - 8))) - 1ull)) : 0ull;
  if (t > 8) { uint64_t k = k2; k *= c2; k = rotl64(k, 33); k *= c1; h2 ^= k; }
  if (t > 0) { uint64_t k = k1; k *= c1; k = rotl64(k, 31); k *= c2; h1 ^= k; }
  h1 ^= (uint64_t)(int64_t)len;
  h2 ^= (uint64_t)(int64_t)len;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  return h1;
}

// Event model of BlockCompressedInputStream (SURVEY.md A.2, 1.131 semantics): a read()
// call that starts exactly where an empty BGZF block follows returns -1; empty blocks
// strictly inside a read are transparent; the hard end H (end of data, or the first block
// that fails to read) ends every read.  decode() issues one read per field.
// ev: the empty blocks' positions in ascending order (binary search; duplicates allowed)
static __device__ __forceinline__ bool empty_at(const uint64_t* __restrict__ ev, uint32_t nev,
                                                uint64_t p) {
  uint32_t lo = 0, hi = nev;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ev[mid] < p) lo = mid + 1;
    else hi = mid;
  }
  return lo < nev && ev[lo] == p;
}

__global__ void k_decode_fixed(const uint8_t* __restrict__ u, uint64_t nrec,
                               const uint64_t* __restrict__ rec_off,
                               const uint64_t* __restrict__ voffset, uint64_t v_end,
                               uint64_t hard_end, int32_t hard_code,
                               const uint64_t* __restrict__ ev, uint32_t nev, int32_t n_ref,
                               int32_t validate_refs, DevColumns c,
                               unsigned long long* __restrict__ first_stop) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrec) return;
  const uint64_t r = rec_off[i];
  // every fixed field read up front (ubuf + slack holds r + 36 for any record start), so one
  // memory round trip follows rec_off instead of two (block_size, then the fields)
  const uint8_t* p = u + r;
  const int32_t bs0 = (int32_t)ld_u32_unaligned(p), ref0 = (int32_t)ld_u32_unaligned(p + 4),
                pos0 = (int32_t)ld_u32_unaligned(p + 8);
  const uint32_t w12 = ld_u32_unaligned(p + 12), w16 = ld_u32_unaligned(p + 16);
  const int32_t lseq0 = (int32_t)ld_u32_unaligned(p + 20), nref0 = (int32_t)ld_u32_unaligned(p + 24),
                npos0 = (int32_t)ld_u32_unaligned(p + 28), tlen0 = (int32_t)ld_u32_unaligned(p + 32);
  int32_t st = ST_OK;
  // split bound (nextKeyValue :173): checked before decode()
  if ((int64_t)voffset[i] >= (int64_t)v_end) {
    st = ST_VEND;
  } else if (empty_at(ev, nev, r)) {
    st = ST_NULL;
  } else if (hard_end < r + 4) {
    st = (hard_code == HBAM_EEOF) ? ST_NULL : hard_code;
  }
  int32_t bs = 0;
  if (st == ST_OK) {
    bs = bs0;
    if (bs < 32) st = HBAM_EFORMAT;
  }
  if (st == ST_OK && nev) {
    // read() calls of decode(): block_size | refID | pos | l_read_name | MAPQ | bin |
    // n_cigar | flag | l_seq | next_refID | next_pos | tlen | rest (only if bs > 32)
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const uint32_t o = k == 0 ? 4 : k == 1 ? 8 : k == 2 ? 12 : k == 3 ? 13 : k == 4 ? 14
                       : k == 5 ? 16 : k == 6 ? 18 : k == 7 ? 20 : k == 8 ? 24 : k == 9 ? 28
                       : k == 10 ? 32 : 36;
      if (k == 11 && bs <= 32) break;
      if (st == ST_OK && r + o <= hard_end && empty_at(ev, nev, r + o)) st = HBAM_EEOF;
    }
  }
  if (st == ST_OK && hard_end < r + 4 + (uint64_t)(uint32_t)bs) st = hard_code;
  int32_t ref = 0, pos = 0, lseq = 0, nref = 0, npos = 0, tlen = 0;
  uint8_t lrn = 0, mapq = 0;
  uint16_t bin = 0, ncig = 0, flag = 0;
  if (st == ST_OK) {
    ref = ref0;
    pos = pos0;
    lrn = (uint8_t)w12;
    mapq = (uint8_t)(w12 >> 8);
    bin = (uint16_t)(w12 >> 16);
    ncig = (uint16_t)w16;
    flag = (uint16_t)(w16 >> 16);
    lseq = lseq0;
    nref = nref0;
    npos = npos0;
    tlen = tlen0;
    if (validate_refs && ((ref != -1 && (ref < 0 || ref >= n_ref)) ||
                          (nref != -1 && (nref < 0 || nref >= n_ref))))
      st = HBAM_EREFID;
  }
  if (st != ST_OK) {
    atomicMin(first_stop, (unsigned long long)i);
    c.status[i] = st;
    c.name_len[i] = 0;
    c.cigar_n[i] = 0;
    c.seq_len[i] = 0;
    c.aux_len[i] = 0;
    return;
  }
  c.status[i] = ST_OK;
  c.block_size[i] = bs;
  c.ref_id[i] = ref;
  c.pos[i] = pos;
  c.l_read_name[i] = lrn;
  c.mapq[i] = mapq;
  c.bin[i] = bin;
  c.n_cigar[i] = ncig;
  c.flag[i] = flag;
  c.l_seq[i] = lseq;
  c.next_ref_id[i] = nref;
  c.next_pos[i] = npos;
  c.tlen[i] = tlen;
  // key: BAMRecordReader.getKey(SAMRecord) :66-96
  const int32_t start = (int32_t)((uint32_t)pos + 1u);
  int64_t key;
  if (!((flag & 4) || ref < 0 || start < 0)) {
    key = (int64_t)((uint64_t)(int64_t)ref << 32 | (uint64_t)(int64_t)pos);
  } else {
    const int32_t h = (int32_t)murmur3_java(u + r + 36, bs - 32);
    key = (int64_t)((uint64_t)0x7fffffffULL << 32 | (uint64_t)(int64_t)h);
  }
  c.key[i] = key;
  // variable-block layout: name | cigar | seq (packed) | qual | aux
  const int64_t var = (int64_t)bs - 32;
  const int64_t fixed_var = (int64_t)lrn + 4 * (int64_t)ncig + ((int64_t)lseq + 1) / 2 + (int64_t)lseq;
  if (lseq < 0 || fixed_var > var) {
    c.layout_ok[i] = 0;
    c.name_len[i] = 0;
    c.cigar_n[i] = 0;
    c.seq_len[i] = 0;
    c.aux_len[i] = 0;
  } else {
    c.layout_ok[i] = 1;
    c.name_len[i] = lrn;
    c.cigar_n[i] = ncig;
    c.seq_len[i] = (uint32_t)lseq;
    c.aux_len[i] = (uint32_t)(var - fixed_var);
  }
}

// Pools: names (l_read_name bytes incl. NUL), CIGAR u32s, SEQ unpacked to
// "=ACMGRSVTWYHKDBN", QUAL raw, AUX raw.  A wave takes a tile of 64 consecutive records (grid-
// stride over tiles).  Each field's segments are cut into 16-byte units (the last unit of a
// segment shorter, written in 8/4/2/1-byte pieces, so a neighbour's bytes in the pool are never
// written); the tile's units are numbered by a wave scan and the lanes take consecutive units,
// so a wave instruction moves ~1 KiB of consecutive pool bytes from a nearly consecutive source.
// Unit size A/B at 5 GB: 8 B 10.1 ms, 16 B 8.3 ms, 32 B 14.2 ms
// (profiles/r03/ab/pools_unit_5g.txt, pools_unit8_5g.txt).
// (r02: one wave per record with byte copies, latency-bound, and a grid of 64 x records threads
// that passed 2^32 above 67 M records; one thread per record with 16-byte copies: 59.7 ms per
// 10 GB shard, every store instruction touching 64 lines.)
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef uint64_t u64_a1 __attribute__((aligned(1)));
// the first n < 16 bytes of v in 8/4/2/1-byte pieces, through a global-address-space pointer
// (global_store_*: a generic pointer made them flat_store_*)
#define HBAM_G __attribute__((address_space(1)))
static __device__ __forceinline__ void st_part_g(HBAM_G uint8_t* d, uint32_t n, u32x4_a1 v) {  // n < 16
  uint64_t lo = (uint64_t)v[0] | (uint64_t)v[1] << 32, hi = (uint64_t)v[2] | (uint64_t)v[3] << 32;
  if (n & 8u) { *(HBAM_G u64_a1*)d = lo; d += 8; lo = hi; }
  if (n & 4u) { *(HBAM_G u32_a1*)d = (uint32_t)lo; d += 4; lo >>= 32; }
  if (n & 2u) { *(HBAM_G u16_a1*)d = (uint16_t)lo; d += 2; lo >>= 16; }
  if (n & 1u) *d = (uint8_t)lo;
}
// 4 SEQ characters of the packed bytes b0 (high nibble first) and b1
static __device__ __forceinline__ uint32_t seq4(uint32_t b0, uint32_t b1) {
  // "=ACMGRSVTWYHKDBN" as two 8-byte halves for v_perm (selector byte = nibble & 7)
  const uint32_t a0 = 0x4d43413du, a1 = 0x56535247u, a2 = 0x48595754u, a3 = 0x4e42444bu;
  const uint32_t n0 = b0 >> 4, n1 = b0 & 15u, n2 = b1 >> 4, n3 = b1 & 15u;
  const uint32_t sel = (n0 & 7u) | (n1 & 7u) << 8 | (n2 & 7u) << 16 | (n3 & 7u) << 24;
  const uint32_t lo = __builtin_amdgcn_perm(a1, a0, sel), hi = __builtin_amdgcn_perm(a3, a2, sel);
  const uint32_t m = ((n0 >> 3) * 0xffu) | ((n1 >> 3) * 0xffu) << 8 | ((n2 >> 3) * 0xffu) << 16 |
                     ((n3 >> 3) * 0xffu) << 24;
  return (lo & ~m) | (hi & m);
}
// 8 SEQ characters of the 4 packed bytes x (byte 0 first, high nibble first): the nibbles spread
// to bytes in order by two v_perm, then the same two-table lookup as seq4 for 4 characters at a
// time, the high-table mask from bit 3 of each nibble as (t << 8) - t
static __device__ __forceinline__ void seq8(uint32_t x, uint32_t& o0, uint32_t& o1) {
  const uint32_t a0 = 0x4d43413du, a1 = 0x56535247u, a2 = 0x48595754u, a3 = 0x4e42444bu;
  const uint32_t lo = x & 0x0f0f0f0fu, hi = (x >> 4) & 0x0f0f0f0fu;
  const uint32_t na = __builtin_amdgcn_perm(hi, lo, 0x01050004u), nb = __builtin_amdgcn_perm(hi, lo, 0x03070206u);
  const uint32_t sa = na & 0x07070707u, sb = nb & 0x07070707u;
  const uint32_t ta = (na >> 3) & 0x01010101u, tb = (nb >> 3) & 0x01010101u;
  const uint32_t ma = (ta << 8) - ta, mb = (tb << 8) - tb;
  o0 = (__builtin_amdgcn_perm(a1, a0, sa) & ~ma) | (__builtin_amdgcn_perm(a3, a2, sa) & ma);
  o1 = (__builtin_amdgcn_perm(a1, a0, sb) & ~mb) | (__builtin_amdgcn_perm(a3, a2, sb) & mb);
}
// The unit -> record mapping without the LDS pipe's shuffles (round 5; the round-4 kernel spent
// ~11 ds_bpermute per 64 units on a 6-step binary search over the lanes' first units plus the
// record's fields, and 7 per field scan: 9.17 -> 8.87 ms at 5 GB, same pools,
// profiles/r05/ab/pools2_dpp_table_5g.txt).  The scans are DPP, each record with units writes
// (source, destination, bytes, first unit) once into LDS at its rank among the tile's records
// with units, and a unit finds its record's rank as a popcount: the records whose first unit lies
// in the 64-unit window are one bit each of a mask (distinct positions), the earlier ones are
// counted by one ballot.  One ds_read_b128 per unit.
// windows per step; A/B at 5 GB, pools ms: 1 9.34, 2 8.57, 3 8.88, 4 8.51
// (profiles/r05/ab/pools_windows_per_step_5g.txt; same pools in every build)
constexpr uint32_t POOLS_U = 4;
static __device__ __forceinline__ uint64_t readlane64(uint64_t x, uint32_t l) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)l) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), (int)l) << 32;
}
// Record-major units: the field-major loop below reads a tile's source lines once
// per field, and a tile's source (64 records, ~22 KB) is evicted from the 4 MB L2 of an XCD (768
// resident waves) before the next field comes to it — FETCH_SIZE counted 2.8 x U for that loop
// (profiles/r05/pmc_kernels.json).  Here a tile's segments (record, field) are numbered in record
// order, so the windows walk the tile's source once, front to back, and are full across field
// ends.  A unit's segment is found in two steps: its record by the record starts' mask (one bit
// per lane, two DPP scans and a ballot per window, as the field-major loop), then its field by
// the record's cumulative unit counts (16-bit, in the record's LDS entry), the segment's entry at
// 64 + 5 x record + field; the five pool bases come from a per-wave LDS table.  (A first form
// found the segment directly, five segment starts per lane in the window mask: 0.3-0.5 ms slower
// at 5 GB, profiles/r05/ab/pools_record_level_mapping_5g.txt.)  Taken for tiles whose records
// are all under 2^16 units (1 MiB); other tiles take the field-major loop.
static __device__ __forceinline__ void pools_tile_rm(const uint8_t* __restrict__ u, const DevColumns& c,
                                                      uint4* segs, uint64_t* pbt, uint32_t lane, uint64_t le,
                                                      uint64_t src, const uint32_t (&L)[5],
                                                      const uint64_t (&d)[5], uint32_t R) {
  uint32_t so[5], cu[5];
  so[0] = 0u;
  so[1] = L[0];
  so[2] = so[1] + L[1];
  so[3] = so[2] + (L[2] + 1u) / 2u;  // packed SEQ
  so[4] = so[3] + L[3];
  cu[0] = 0u;
#pragma unroll
  for (int f = 1; f < 5; ++f) cu[f] = cu[f - 1] + ((L[f - 1] + 15u) >> 4);
  const uint32_t incl = wave_scan_dpp(R), E = incl - R, T = wave_last(incl);
  if (T == 0u) return;
  const uint64_t mh = __ballot(R != 0u);
  const uint32_t first = (uint32_t)__builtin_ctzll(mh);
  const uint64_t sb = readlane64(src, first);
  uint64_t db[5];
#pragma unroll
  for (int f = 0; f < 5; ++f) db[f] = readlane64(d[f], first);
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");  // the previous tile's reads of segs / pbt precede these writes
  if (R != 0u) {
    const uint32_t rk = lane_rank(mh);
    segs[rk] = make_uint4(E, (uint32_t)(src - sb), cu[1] | cu[2] << 16, cu[3] | cu[4] << 16);
#pragma unroll
    for (int f = 0; f < 5; ++f)
      segs[64u + 5u * rk + (uint32_t)f] = make_uint4((uint32_t)(d[f] - db[f]), L[f], so[f], cu[f]);
  }
  if (lane < 5u) {
    uint8_t* const b = lane == 0u ? c.names : lane == 1u ? (uint8_t*)c.cigars : lane == 2u ? c.seq
                     : lane == 3u ? c.qual : c.aux;
    const uint64_t dbl = lane == 0u ? db[0] : lane == 1u ? db[1] : lane == 2u ? db[2] : lane == 3u ? db[3] : db[4];
    pbt[lane] = (uint64_t)(uintptr_t)(b + dbl);
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  const uint8_t* const sbase = u + sb;
  for (uint32_t q0 = 0; q0 < T; q0 += 64 * POOLS_U) {
    u32x4_t raw[POOLS_U];
    const uint8_t* sp[POOLS_U];
    uint8_t* dp[POOLS_U];
    uint32_t nn[POOLS_U], fs[POOLS_U];
#pragma unroll
    for (uint32_t w = 0; w < POOLS_U; ++w) {
      nn[w] = 0;
      fs[w] = 0;
      dp[w] = (uint8_t*)sbase;  // (never stored through: nn = 0)
      sp[w] = sbase;
      const uint32_t qw = q0 + 64u * w;
      if (qw >= T) continue;  // wave-uniform
      const uint32_t q = qw + lane;
      const uint32_t pos = E - qw;
      const bool inwin = R != 0u && E >= qw && pos < 64u;
      const uint32_t blo = (inwin && pos < 32u) ? 1u << pos : 0u;
      const uint32_t bhi = (inwin && pos >= 32u) ? 1u << (pos - 32u) : 0u;
      const uint64_t M = (uint64_t)wave_last(wave_scan_dpp(bhi)) << 32 | wave_last(wave_scan_dpp(blo));
      const uint32_t c0 = (uint32_t)__popcll(__ballot(R != 0u && E < qw));
      if (q < T) {
        const uint32_t rk = c0 + (uint32_t)__popcll(M & le) - 1u;
        const uint4 A = segs[rk];
        const uint32_t dq = q - A.x;
        const uint32_t f = (dq >= (A.z & 0xffffu) ? 1u : 0u) + (dq >= (A.z >> 16) ? 1u : 0u) +
                           (dq >= (A.w & 0xffffu) ? 1u : 0u) + (dq >= (A.w >> 16) ? 1u : 0u);
        const uint4 S = segs[64u + 5u * rk + f];
        const uint32_t j = dq - S.w, len = S.y;
        uint32_t n = len - 16u * j;
        const uint32_t sbk = (n < 16u && len >= 16u && (f != 2u || (n & 1u) == 0u)) ? 16u - n : 0u;
        n += sbk;
        nn[w] = n;
        dp[w] = (uint8_t*)(uintptr_t)pbt[f] + S.x + 16u * j - sbk;
        sp[w] = sbase + A.y + S.z + (f == 2u ? 8u * j - sbk / 2u : 16u * j - sbk);
        fs[w] = f;
      }
    }
    asm volatile("global_load_dwordx4 %0, %4, off\n\tglobal_load_dwordx4 %1, %5, off\n\t"
                 "global_load_dwordx4 %2, %6, off\n\tglobal_load_dwordx4 %3, %7, off\n\ts_waitcnt vmcnt(0)"
                 : "=&v"(raw[0]), "=&v"(raw[1]), "=&v"(raw[2]), "=&v"(raw[3])
                 : "v"(sp[0]), "v"(sp[1]), "v"(sp[2]), "v"(sp[3]) : "memory");
#pragma unroll
    for (uint32_t w = 0; w < POOLS_U; ++w) {
      if (q0 + 64u * w >= T) break;  // wave-uniform
      u32x4_a1 v = u32x4_a1{raw[w][0], raw[w][1], raw[w][2], raw[w][3]};
      if (__ballot(fs[w] == 2u) != 0ull) {  // a SEQ unit in the window: 8 packed bytes -> 16 chars
        const bool sq = fs[w] == 2u;
        uint32_t c0s, c1s, c2s, c3s;  // (seq4 per 4 characters: 0.27-0.33 ms slower per 5 GB,
        seq8(raw[w][0], c0s, c1s);     // profiles/r05/ab/pools_seq8_5g.txt)
        seq8(raw[w][1], c2s, c3s);
        v[0] = sq ? c0s : v[0];
        v[1] = sq ? c1s : v[1];
        v[2] = sq ? c2s : v[2];
        v[3] = sq ? c3s : v[3];
      }
      HBAM_G uint8_t* const gd = (HBAM_G uint8_t*)dp[w];
      if (nn[w] >= 16u) *(HBAM_G u32x4_a1*)gd = v;
      else if (nn[w] != 0u) st_part_g(gd, nn[w], v);
    }
  }
}
__global__ __launch_bounds__(256) void k_decode_pools(const uint8_t* __restrict__ u, uint64_t nrec,
                                                       const uint64_t* __restrict__ rec_off,
                                                       DevColumns c) {
  __shared__ uint4 s_recs[4][384];
  __shared__ uint64_t s_pb[4][8];
  const uint32_t lane = threadIdx.x & 63u;
  uint4* const recs = s_recs[threadIdx.x >> 6];
  const uint64_t ntiles = (nrec + 63) / 64;
  const uint64_t wstride = (uint64_t)gridDim.x * (blockDim.x / 64);
  const uint64_t le = lane == 63u ? ~0ull : ((2ull << lane) - 1ull);  // lanes <= this one
  for (uint64_t t = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); t < ntiles; t += wstride) {
    const uint64_t r = t * 64 + lane;
    uint32_t nl = 0, nc = 0, ls = 0, na = 0;
    uint64_t src = 0, o_name = 0, o_cig = 0, o_seq = 0, o_aux = 0;
    if (r < nrec && c.layout_ok[r]) {
      src = rec_off[r] + 36;
      nl = c.name_len[r];
      nc = c.cigar_n[r];
      ls = c.seq_len[r];
      na = c.aux_len[r];
      o_name = c.name_off[r];
      o_cig = c.cigar_off[r];
      o_seq = c.seq_off[r];
      o_aux = c.aux_off[r];
    }
    {
      const uint32_t L[5] = {nl, 4u * nc, ls, ls, na};
      const uint64_t d[5] = {o_name, 4 * o_cig, o_seq, o_seq, o_aux};
      uint32_t R = 0u;
      bool big = false;
#pragma unroll
      for (int f = 0; f < 5; ++f) {
        R += (L[f] + 15u) >> 4;
        big |= L[f] >= (1u << 20);
      }
      if (__ballot(big || R >= (1u << 16)) == 0ull) {  // wave-uniform
        pools_tile_rm(u, c, recs, s_pb[threadIdx.x >> 6], lane, le, src, L, d, R);
        continue;
      }
    }
#pragma unroll 1
    for (uint32_t f = 0; f < 5; ++f) {
      uint32_t len;
      uint64_t s0, d0;
      uint8_t* base;
      if (f == 0) { len = nl; s0 = src; d0 = o_name; base = c.names; }
      else if (f == 1) { len = 4u * nc; s0 = src + nl; d0 = 4 * o_cig; base = (uint8_t*)c.cigars; }
      else if (f == 2) { len = ls; s0 = src + nl + 4u * nc; d0 = o_seq; base = c.seq; }
      else if (f == 3) { len = ls; s0 = src + nl + 4u * nc + (ls + 1u) / 2u; d0 = o_seq; base = c.qual; }
      else { len = na; s0 = src + nl + 4u * nc + (ls + 1u) / 2u + ls; d0 = o_aux; base = c.aux; }
      const uint32_t units = (len + 15u) >> 4;
      const uint32_t incl = wave_scan_dpp(units), excl = incl - units, total = wave_last(incl);
      if (total == 0u) continue;
      const bool has = units != 0u;
      const uint64_t mh = __ballot(has);
      const uint32_t first = (uint32_t)__builtin_ctzll(mh);
      const uint64_t sb = readlane64(s0, first), db = readlane64(d0, first);
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");  // the previous field's reads of recs precede these writes
      if (has) recs[lane_rank(mh)] = make_uint4((uint32_t)(s0 - sb), (uint32_t)(d0 - db), len, excl);
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");  // (one wave: its LDS operations run in issue order)
      uint8_t* const dbase = base + db;
      const uint8_t* const sbase = u + sb;
      // POOLS_U windows per step, their loads issued back to back before any store.  With
      // one window per step the compiler puts s_waitcnt vmcnt(0) ahead of each load (the address
      // is built by VALU writes into registers that held the last store's data, which the store
      // reads late), so every step paid a load round trip plus a store acknowledgement.  The U
      // loads and their wait are ONE asm statement (lanes and windows without a unit read a valid
      // dummy address): nothing the compiler schedules can touch the destinations between a load
      // and its data (a wait in a separate statement let it copy the registers before the data
      // had landed), and no load is left in flight after the statement.
      for (uint32_t q0 = 0; q0 < total; q0 += 64 * POOLS_U) {
        u32x4_t raw[POOLS_U];
        const uint8_t* sp[POOLS_U];
        uint8_t* dp[POOLS_U];
        uint32_t nn[POOLS_U];
#pragma unroll
        for (uint32_t w = 0; w < POOLS_U; ++w) {
          nn[w] = 0;
          dp[w] = dbase;
          sp[w] = sbase;
          const uint32_t qw = q0 + 64u * w;
          if (qw >= total) continue;  // wave-uniform
          const uint32_t q = qw + lane;
          const uint32_t pos = excl - qw;
          const bool inwin = has && excl >= qw && pos < 64u;
          const uint32_t blo = (inwin && pos < 32u) ? 1u << pos : 0u;
          const uint32_t bhi = (inwin && pos >= 32u) ? 1u << (pos - 32u) : 0u;
          const uint64_t M = (uint64_t)wave_last(wave_scan_dpp(bhi)) << 32 | wave_last(wave_scan_dpp(blo));
          const uint32_t c0 = (uint32_t)__popcll(__ballot(has && excl < qw));
          if (q < total) {
            const uint4 rr = recs[c0 + (uint32_t)__popcll(M & le) - 1u];
            const uint32_t k = q - rr.w;
            nn[w] = rr.z - 16u * k;
            dp[w] = dbase + rr.y + 16u * k;
            sp[w] = sbase + rr.x + (f == 2 ? 8u : 16u) * k;
          }
        }
        asm volatile("global_load_dwordx4 %0, %4, off\n\tglobal_load_dwordx4 %1, %5, off\n\t"
                     "global_load_dwordx4 %2, %6, off\n\tglobal_load_dwordx4 %3, %7, off\n\ts_waitcnt vmcnt(0)"
                     : "=&v"(raw[0]), "=&v"(raw[1]), "=&v"(raw[2]), "=&v"(raw[3])
                     : "v"(sp[0]), "v"(sp[1]), "v"(sp[2]), "v"(sp[3]) : "memory");
#pragma unroll
        for (uint32_t w = 0; w < POOLS_U; ++w) {
          if (q0 + 64u * w >= total) break;  // wave-uniform
          u32x4_a1 v;
          if (f == 2) {
            const uint64_t qq = (uint64_t)raw[w][0] | (uint64_t)raw[w][1] << 32;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              v[j] = seq4((uint32_t)(qq >> (16 * j)) & 0xffu, (uint32_t)(qq >> (16 * j + 8)) & 0xffu);
          } else {
            v = u32x4_a1{raw[w][0], raw[w][1], raw[w][2], raw[w][3]};
          }
          HBAM_G uint8_t* const gd = (HBAM_G uint8_t*)dp[w];
          if (nn[w] >= 16u) *(HBAM_G u32x4_a1*)gd = v;
          else if (nn[w] != 0u) st_part_g(gd, nn[w], v);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// scans (u32 -> u64 exclusive), 3-phase reduce-then-scan
// ------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(SCAN_WG) void k_scan_reduce(const T* __restrict__ in, uint64_t n,
                                                         uint64_t* __restrict__ partial) {
  __shared__ uint64_t s[SCAN_WG];
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
  uint64_t acc = 0;
  for (uint32_t k = threadIdx.x; k < SCAN_TILE; k += SCAN_WG) {
    const uint64_t j = base + k;
    if (j < n) acc += (uint64_t)in[j];
  }
  s[threadIdx.x] = acc;
  __syncthreads();
  for (uint32_t o = SCAN_WG / 2; o; o >>= 1) {
    if (threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = s[0];
}

__global__ __launch_bounds__(SCAN_WG) void k_scan_partials(uint64_t* __restrict__ partial,
                                                           uint64_t n, uint64_t* __restrict__ total) {
  __shared__ uint64_t s[SCAN_WG];
  uint64_t carry = 0;
  for (uint64_t base = 0; base < n; base += SCAN_WG) {
    const uint64_t j = base + threadIdx.x;
    const uint64_t v = j < n ? partial[j] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t o = 1; o < SCAN_WG; o <<= 1) {
      const uint64_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
      __syncthreads();
      s[threadIdx.x] += t;
      __syncthreads();
    }
    if (j < n) partial[j] = carry + s[threadIdx.x] - v;
    const uint64_t tot = s[SCAN_WG - 1];
    __syncthreads();
    carry += tot;
  }
  if (threadIdx.x == 0) *total = carry;
}

template <typename T>
__global__ __launch_bounds__(SCAN_WG) void k_scan_apply(const T* __restrict__ in, uint64_t n,
                                                        const uint64_t* __restrict__ partial,
                                                        uint64_t* __restrict__ out) {
  __shared__ uint64_t s[SCAN_WG];
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
  uint64_t carry = partial[blockIdx.x];
  for (uint32_t t0 = 0; t0 < SCAN_TILE; t0 += SCAN_WG) {
    const uint64_t j = base + t0 + threadIdx.x;
    const uint64_t v = j < n ? (uint64_t)in[j] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t o = 1; o < SCAN_WG; o <<= 1) {
      const uint64_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
      __syncthreads();
      s[threadIdx.x] += t;
      __syncthreads();
    }
    if (j < n) out[j] = carry + s[threadIdx.x] - v;
    const uint64_t tot = s[SCAN_WG - 1];
    __syncthreads();
    carry += tot;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = carry;
}

// explicit instantiations used by the runtime
// ---- the four pool-length scans at once (names, CIGAR, SEQ/QUAL, AUX: u32 -> u64 exclusive)
// Three launches for the four arrays instead of twelve, and a thread takes 16 consecutive
// elements of each array (four 16-byte loads) with the block scan on registers and one LDS pass
// instead of k_scan_apply's sixteen LDS Hillis-Steele rounds per tile.  The arrays hold n + 16
// readable elements (fill_columns: n + 1 plus the 64-byte pad), so a tile's tail needs no guard on
// its loads, only on the values.
constexpr uint32_t SCAN4_PER = 16, SCAN4_TILE = 256u * SCAN4_PER;
struct Scan4In {
  const uint32_t* a[4];
};
struct Scan4Out {
  uint64_t* o[4];
};
static __device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, o), hi = __shfl_xor((uint32_t)(v >> 32), o);
    v += (uint64_t)hi << 32 | lo;
  }
  return v;
}
static __device__ __forceinline__ void scan4_load(const uint32_t* __restrict__ a, uint64_t e0, uint64_t n,
                                                  uint32_t (&v)[SCAN4_PER]) {
  const bool any = e0 < n;  // a thread past the end loads nothing
#pragma unroll
  for (uint32_t k = 0; k < SCAN4_PER; k += 4) {
    const uint4 q = any ? *(const uint4*)(a + e0 + k) : make_uint4(0, 0, 0, 0);
    v[k] = e0 + k < n ? q.x : 0u;
    v[k + 1] = e0 + k + 1 < n ? q.y : 0u;
    v[k + 2] = e0 + k + 2 < n ? q.z : 0u;
    v[k + 3] = e0 + k + 3 < n ? q.w : 0u;
  }
}
__global__ __launch_bounds__(256) void k_scan4_reduce(Scan4In in, uint64_t n, uint64_t* __restrict__ partial,
                                                      uint32_t tiles) {
  __shared__ uint64_t s[4][4];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  const uint64_t e0 = (uint64_t)blockIdx.x * SCAN4_TILE + (uint64_t)tid * SCAN4_PER;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t v[SCAN4_PER];
    scan4_load(in.a[q], e0, n, v);
    uint64_t t = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN4_PER; ++k) t += v[k];
    t = wave_sum_u64(t);
    if (lane == 0) s[q][w] = t;
  }
  __syncthreads();
  if (tid < 4) partial[(uint64_t)tid * tiles + blockIdx.x] = s[tid][0] + s[tid][1] + s[tid][2] + s[tid][3];
}
// one workgroup per array: exclusive scan of its tile sums in place; out[n] = the array's total
__global__ __launch_bounds__(256) void k_scan4_partials(uint64_t* __restrict__ partial, uint32_t tiles,
                                                        Scan4Out out, uint64_t n) {
  __shared__ uint64_t s[4];
  const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  uint64_t* p = partial + (uint64_t)q * tiles;
  uint64_t carry = 0;
  for (uint32_t b0 = 0; b0 < tiles; b0 += 256) {
    const uint32_t j = b0 + tid;
    const uint64_t v = j < tiles ? p[j] : 0;
    uint64_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t lo = __shfl_up((uint32_t)incl, o), hi = __shfl_up((uint32_t)(incl >> 32), o);
      if ((int)lane >= o) incl += (uint64_t)hi << 32 | lo;
    }
    if (lane == 63) s[w] = incl;
    __syncthreads();
    uint64_t wb = 0;
    for (uint32_t k = 0; k < w; ++k) wb += s[k];
    const uint64_t tot = s[0] + s[1] + s[2] + s[3];
    if (j < tiles) p[j] = carry + wb + incl - v;
    carry += tot;
    __syncthreads();
  }
  if (tid == 0) out.o[q][n] = carry;
}
__global__ __launch_bounds__(256) void k_scan4_apply(Scan4In in, uint64_t n, const uint64_t* __restrict__ partial,
                                                     uint32_t tiles, Scan4Out out) {
  __shared__ uint64_t s[4][4];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  const uint64_t e0 = (uint64_t)blockIdx.x * SCAN4_TILE + (uint64_t)tid * SCAN4_PER;
  uint64_t base[4], tt[4];
  uint32_t v[4][SCAN4_PER];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    scan4_load(in.a[q], e0, n, v[q]);
    uint64_t t = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN4_PER; ++k) t += v[q][k];
    uint64_t incl = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t lo = __shfl_up((uint32_t)incl, o), hi = __shfl_up((uint32_t)(incl >> 32), o);
      if ((int)lane >= o) incl += (uint64_t)hi << 32 | lo;
    }
    if (lane == 63) s[q][w] = incl;
    tt[q] = incl - t;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint64_t wb = partial[(uint64_t)q * tiles + blockIdx.x];
    for (uint32_t k = 0; k < w; ++k) wb += s[q][k];
    base[q] = wb + tt[q];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint64_t run = base[q];
    uint64_t r[SCAN4_PER];
#pragma unroll
    for (uint32_t k = 0; k < SCAN4_PER; ++k) {
      r[k] = run;
      run += v[q][k];
    }
    uint64_t* o = out.o[q] + e0;
    if (e0 + SCAN4_PER <= n) {
#pragma unroll
      for (uint32_t k = 0; k < SCAN4_PER; k += 2) *(ulonglong2*)(o + k) = make_ulonglong2(r[k], r[k + 1]);
    } else {
#pragma unroll
      for (uint32_t k = 0; k < SCAN4_PER; ++k)
        if (e0 + k < n) o[k] = r[k];
    }
  }
}

template __global__ void k_scan_reduce<uint32_t>(const uint32_t*, uint64_t, uint64_t*);
template __global__ void k_scan_apply<uint32_t>(const uint32_t*, uint64_t, const uint64_t*, uint64_t*);

}  // namespace hbam
