// hbam_capi.hip — host runtime + C ABI (include/hbam.h) of the MI355X BAM read path.
//
// One context = one device + one HIP stream + grow-only device work buffers.  The
// per-split pipeline (hbam_decode_split) is:
//   K1 scan chunks -> gather -> verify chain      (BGZF block table, device)
//   K2 inflate (+ K2b CRC)                        (lane per block, device)
//   K5 entry/walk/stitch/fix/emit                 (record starts + voffsets, device)
//   K6/K7/K8 decode fixed fields, status, keys    (device)
//   pools (names/CIGAR/SEQ/QUAL/AUX)              (device)
// The host only decides control flow from a few downloaded scalars (chain end,
// first bad block, first stop record) — the reference's exception semantics.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "hbam_internal.h"
#include "hbam_kernels.hip"
#include "hbam_guess.hip"
#include "hbam_bcf.hip"
#include "hbam_sort.hip"
#include "hbam_deflate.hip"

using namespace hbam;

constexpr uint64_t GUESS_BATCH = 16384;  // guesses per launch (~66 KiB of scratch + the window cache
                                         // each); env HBAM_GUESS_BATCH overrides (tests: multi-batch)

namespace {

struct Buf {
  void* p = nullptr;
  size_t cap = 0;
};

enum BufId {
  B_COMP,
  B_CHUNK_CNT,
  B_CHUNK_BASE,
  B_CHUNK_POS,
  B_CAND,
  B_BLK,
  B_UOFF,
  B_ISZ32,
  B_UBUF,
  B_LENS,
  B_BITMAP,
  B_TAILS,
  B_EDGE,
  B_RETRY,
  B_INFST,
  B_CRC,
  B_ENTRY,
  B_EXIT,
  B_REL,
  B_COUNT,
  B_RECBASE,
  B_RECOFF,
  B_VOFF,
  B_SMALL,
  B_PARTIAL,
  B_EVENTS,
  B_EVFLAG,
  B_EVPOS,
  B_BADLIST,
  B_MARK,
  // columns
  B_C_STATUS,
  B_C_BS,
  B_C_REF,
  B_C_POS,
  B_C_LRN,
  B_C_MAPQ,
  B_C_BIN,
  B_C_NCIG,
  B_C_FLAG,
  B_C_LSEQ,
  B_C_NREF,
  B_C_NPOS,
  B_C_TLEN,
  B_C_KEY,
  B_C_LAYOUT,
  B_C_NAMELEN,
  B_C_CIGN,
  B_C_SEQLEN,
  B_C_AUXLEN,
  B_C_NAMEOFF,
  B_C_CIGOFF,
  B_C_SEQOFF,
  B_C_AUXOFF,
  B_C_NAMES,
  B_C_CIGARS,
  B_C_SEQ,
  B_C_QUAL,
  B_C_AUX,
  // guesser window cache
  B_G_WORK,
  B_G_CN,
  B_G_CBASE,
  B_G_SLOTS,
  B_G_CPOS,
  B_G_CBLK,
  B_G_CISZ,
  B_G_CNEFF,
  B_G_CUOFF,
  B_G_CUBUF,
  B_G_CST,
  B_G_CCRC,
  B_G_WIN,  // caller-gathered guess windows staged from the host
  B_S_UK0,
  B_S_UK1,
  B_S_V0,
  B_S_V1,
  B_S_CNT,
  B_S_OFF,
  B_S_HIST,
  B_S_LENS,
  B_S_PERM,
  B_S_RECOFF,
  B_S_BOUNDS,
  B_M_MAP,  // multi-input Sort: merged index per input index
  B_M_ERR,
  B_DF_SRC,
  B_DF_TOK,
  B_DF_NTOK,
  B_DF_FREQ,
  B_DF_CRC,
  B_DF_SLOTS,
  B_DF_CSIZE,
  B_DF_OFF,
  B_DF_DST,
  // read-name / CIGAR keyed consumers (hbam_consumers.hip)
  B_F4_CNT,
  B_F4_OFF,
  B_F4_ERR,
  B_F4_KEY,
  B_F4_BEG,
  B_F4_END,
  B_F4_REV,
  B_F4_REC,
  B_F4_NKEY,
  B_F4_NP,
  B_F4_NTMP,
  B_F4_MM,
  B_F4_PERM,
  B_F4_GST,
  B_F4_GCNT,
  B_F4_GOUT,
  B_F4_SRC,
  B_F4_MATE,
  B_F4_ROLE,
  B_F4_LENS,
  B_F4_OOFF,
  B_F4_PAY,
  // BCF read path (hbam_bcf_api.hip)
  B_BCF_COLS,
  B_BCF_SCRATCH,
  // Sort exchange over RCCL (hbam_comm.hip): receive buffers, counts, samples
  B_X_KEY,
  B_X_VOFF,
  B_X_BS,
  B_X_PAY,
  B_X_CNT,
  B_X_SAMP,
  // multi-input Sort: read-/program-group rewrite (hbam_groups.hip)
  B_G_TAB,
  B_G_LENS,
  B_G_ERR,
  B_G_CODES,
  B_G_OOFF,
  B_G_BS,
  B_G_PAY,
  B_RH_RECOFF,  // hbam_records_to_host: rec_off rebased to the copied record bytes
  B_COUNT_ALL
};

}  // namespace

// inflate slices on two streams; A/B at 10 GB: 1 -> 163.4 ms, 2 -> 161.5, 4 -> 166.5, 8 -> 164.5
// (Huffman + LZ77); env HBAM_INFLATE_SLICES overrides
constexpr uint32_t INFLATE_SLICES = 1;
constexpr uint32_t MAX_SLICES = 16;
// Huffman pass by k_inflate_wave (a wave per block) for calls of up to this many BGZF blocks,
// by k_inflate_tokens (a lane per block) above: the lane pass needs ~131k blocks (2 waves x 64
// lanes x 1,024 SIMDs) to fill the chip, the wave pass fills it from a few thousand but costs
// more per block.  Huffman ms, lane vs wave: 1 GB 16.8 / 9.5, 2 GB 20.8 / 18.2, 3 GB 21.5 / 27.0,
// 5 GB 33.8 / 44.7, 10 GB 60 / 88.9 (profiles/r04/ab/huffman_wave_vs_lane_by_size.txt)
// env HBAM_WAVE_MAX_BLOCKS overrides (tests, A/B)
constexpr uint64_t WAVE_MAX_BLOCKS = 90000;
struct hbam_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hbam_opts opts{};
  std::string err;
  Buf bufs[B_COUNT_ALL];
  hipStream_t stream2 = nullptr;  // LZ77 pass of slice s beside the Huffman pass of slice s+1
  hipEvent_t ev[16];
  hipEvent_t slice_ev[MAX_SLICES + 1];
  uint32_t inflate_slices = INFLATE_SLICES;  // env HBAM_INFLATE_SLICES overrides (A/B)
  uint64_t wave_max_blocks = WAVE_MAX_BLOCKS;  // env HBAM_WAVE_MAX_BLOCKS overrides (tests, A/B)
  bool slices_forced = false;                     // ... and then applies to small calls too
  hbam_timing timing{};
  uint64_t* pinned_small = nullptr;  // host pinned scalars
  uint64_t guess_batch = GUESS_BATCH;  // env HBAM_GUESS_BATCH overrides (tests: multi-batch)
  uint8_t* rec_host = nullptr;  // hbam_records_to_host: pinned, grow-only
  size_t rec_host_cap = 0;
  std::vector<hbam_comm*> comms;  // communicators tied to this context (hbam_comm.hip)
};

namespace {

int set_err(hbam_ctx* c, int code, const char* fmt, ...) {
  char b[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(b, sizeof b, fmt, ap);
  va_end(ap);
  if (c) c->err = b;
  return code;
}

#define HIPCHK(ctx, x)                                                                      \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess)                                                                   \
      return set_err((ctx), HBAM_EDEVICE, "%s:%d %s: %s", __FILE__, __LINE__, #x,           \
                     hipGetErrorString(e_));                                                \
  } while (0)

template <typename T>
int ensure(hbam_ctx* c, BufId id, size_t count, T** out) {
  size_t bytes = count * sizeof(T) + 64;
  Buf& b = c->bufs[id];
  if (b.cap < bytes) {
    size_t want = std::max(bytes, b.cap + b.cap / 2);  // grow geometrically
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    hipError_t e = hipMalloc(&b.p, want);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      e = hipMalloc(&b.p, bytes);
      want = bytes;
      if (e != hipSuccess) {
        (void)hipGetLastError();
        b.p = nullptr;
        return set_err(c, HBAM_ENOMEM, "hipMalloc(%zu) failed for buffer %d", bytes, (int)id);
      }
    }
    b.cap = want;
  }
  *out = (T*)b.p;
  return HBAM_OK;
}

float ev_ms(hbam_ctx* c, int a, int b);
inline uint32_t grid_for(uint64_t n, uint32_t wg) { return (uint32_t)((n + wg - 1) / wg); }

// stream-ordered synchronous copy (the context stream is non-blocking: a plain hipMemcpy
// on the null stream would not wait for its kernels)
hipError_t copy_sync(hbam_ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind k) {
  if (!bytes) return hipSuccess;
  hipError_t e = hipMemcpyAsync(dst, src, bytes, k, c->stream);
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(c->stream);
}

// exclusive scan of n u32 values -> out[0..n] (out[n] = total); returns total via host
template <typename T>
int scan_exclusive(hbam_ctx* c, const T* in, uint64_t n, uint64_t* out, uint64_t* total_host) {
  const uint64_t tiles = std::max<uint64_t>(1, (n + SCAN_TILE - 1) / SCAN_TILE);
  uint64_t* partial;
  int rc = ensure(c, B_PARTIAL, tiles + 1, &partial);
  if (rc) return rc;
  k_scan_reduce<T><<<(uint32_t)tiles, SCAN_WG, 0, c->stream>>>(in, n, partial);
  k_scan_partials<<<1, SCAN_WG, 0, c->stream>>>(partial, tiles, partial + tiles);
  k_scan_apply<T><<<(uint32_t)tiles, SCAN_WG, 0, c->stream>>>(in, n, partial, out);
  HIPCHK(c, hipGetLastError());
  if (total_host) {
    HIPCHK(c, hipMemcpyAsync(c->pinned_small, out + n, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *total_host = c->pinned_small[0];
  }
  return HBAM_OK;
}

inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | p[1] << 8); }
inline int32_t rd32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 |
                   (uint32_t)p[3] << 24);
}

// [htsjdk] BCIS.readBlock + BlockGunzipper header checks for a block that the device
// chain does not accept, from up to 26 bytes at its position (`avail` bytes exist).
int readblock_error(const uint8_t* h, uint64_t avail) {
  if (avail == 0) return HBAM_EEOF;      // clean end of data
  if (avail < 18) return HBAM_ERUNTIMEIO; // IOException "Premature end of file" (wrapped)
  const uint32_t blen = (uint32_t)rd16(h + 16) + 1u;
  if (blen < 18) return HBAM_ERUNTIMEIO;  // IOException "Unexpected compressed block length"
  if (blen > avail) return HBAM_ETRUNC;   // FileTruncatedException
  // inflateBlock: ISIZE < 0 -> RuntimeIOException; unzipBlock header checks
  const int32_t isize = rd32(h + blen - 4);
  if (isize < 0) return HBAM_ERUNTIMEIO;
  if (!(h[0] == 0x1f && h[1] == 0x8b && h[2] == 8 && h[3] == 4)) return HBAM_EFORMAT;
  if (rd16(h + 10) != 6) return HBAM_EFORMAT;
  return HBAM_EFORMAT;
}

struct Chain {
  std::vector<BlockRec> blocks;  // host copy only when the fast path fails
  uint64_t nb = 0;
  int32_t end_code = HBAM_EEOF;  // what reading past the last block raises
  uint64_t end_pos = 0;          // comp offset where the chain ends
};

// K1: block table of the chain starting at comp offset `start` (must be a block start).
// Device-resident result in B_BLK (nb entries).  end_code: HBAM_EEOF for a clean end of
// file, a readBlock error code, or HBAM_EMORE when the window ends mid-chain.
int build_chain(hbam_ctx* c, const uint8_t* dcomp, uint64_t comp_len, uint64_t start,
                bool window_is_file_end, Chain* ch) {
  ch->nb = 0;
  if (start >= comp_len) {
    ch->end_code = window_is_file_end ? HBAM_EEOF : HBAM_EMORE;
    ch->end_pos = start;
    return HBAM_OK;
  }
  const uint64_t span = comp_len - start;
  const uint64_t nchunks = (span + SCAN_CHUNK - 1) / SCAN_CHUNK;
  uint32_t* chunk_cnt;
  uint64_t *chunk_base, *chunk_pos, *cand, *small;
  BlockRec* blk;
  int rc;
  if ((rc = ensure(c, B_CHUNK_CNT, nchunks, &chunk_cnt))) return rc;
  if ((rc = ensure(c, B_CHUNK_BASE, nchunks + 1, &chunk_base))) return rc;
  if ((rc = ensure(c, B_CHUNK_POS, nchunks * SCAN_CAP, &chunk_pos))) return rc;
  if ((rc = ensure(c, B_SMALL, 16, &small))) return rc;
  HIPCHK(c, hipMemsetAsync(small, 0, 16 * 8, c->stream));
  uint32_t* overflow = (uint32_t*)small;
  uint32_t* nbad = (uint32_t*)small + 1;
  k_scan_chunks<<<(uint32_t)nchunks, 256, 0, c->stream>>>(dcomp, start, comp_len, chunk_cnt,
                                                          chunk_pos, overflow);
  HIPCHK(c, hipGetLastError());
  uint64_t ncand = 0;
  if ((rc = scan_exclusive<uint32_t>(c, chunk_cnt, nchunks, chunk_base, &ncand))) return rc;
  if ((rc = ensure(c, B_CAND, ncand + 1, &cand))) return rc;
  if ((rc = ensure(c, B_BLK, ncand + 1, &blk))) return rc;
  k_gather_cands<<<grid_for(nchunks, 256), 256, 0, c->stream>>>(chunk_cnt, chunk_base, chunk_pos,
                                                                nchunks, cand);
  if (ncand)
    k_verify_chain<<<grid_for(ncand, 256), 256, 0, c->stream>>>(dcomp, cand, ncand, comp_len,
                                                                 blk, nbad);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(c->pinned_small, small, 16, hipMemcpyDeviceToHost, c->stream));
  // the chain's ends in the same round trip (used when no chunk overflowed)
  if (ncand) {
    HIPCHK(c, hipMemcpyAsync(c->pinned_small + 8, cand, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->pinned_small + 10, blk + (ncand - 1), sizeof(BlockRec), hipMemcpyDeviceToHost,
                             c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint32_t ovf = ((uint32_t*)c->pinned_small)[0];
  uint32_t bad = ((uint32_t*)c->pinned_small)[1];
  bool ends_known = ovf == 0;
  if (ovf) {
    // more than SCAN_CAP candidates in some chunk (blocks of < 1 KiB compressed, or data full
    // of magic patterns): the exact two-pass scan writes the whole candidate list
    k_scan_count<<<(uint32_t)nchunks, 256, 0, c->stream>>>(dcomp, start, comp_len, chunk_cnt);
    HIPCHK(c, hipGetLastError());
    if ((rc = scan_exclusive<uint32_t>(c, chunk_cnt, nchunks, chunk_base, &ncand))) return rc;
    if ((rc = ensure(c, B_CAND, ncand + 1, &cand))) return rc;
    if ((rc = ensure(c, B_BLK, ncand + 1, &blk))) return rc;
    HIPCHK(c, hipMemsetAsync(small, 0, 16 * 8, c->stream));
    k_scan_write<<<(uint32_t)nchunks, 256, 0, c->stream>>>(dcomp, start, comp_len, chunk_base, cand);
    if (ncand)
      k_verify_chain<<<grid_for(ncand, 256), 256, 0, c->stream>>>(dcomp, cand, ncand, comp_len,
                                                                   blk, nbad);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(c->pinned_small, small, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    bad = ((uint32_t*)c->pinned_small)[1];
  }
  // download candidate list only if the fast path failed or to check the ends
  uint64_t first = ~0ULL;
  BlockRec last{};
  if (ncand) {
    if (!ends_known) {
      HIPCHK(c, hipMemcpyAsync(c->pinned_small + 8, cand, 8, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->pinned_small + 10, blk + (ncand - 1), sizeof(BlockRec),
                               hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    first = c->pinned_small[8];
    memcpy(&last, c->pinned_small + 10, sizeof last);
  }
  uint8_t hdr[32];
  auto classify_end = [&](uint64_t pos) -> int32_t {
    const uint64_t avail = comp_len - pos;
    memset(hdr, 0, sizeof hdr);
    const uint64_t nget = std::min<uint64_t>(avail, 32);
    if (nget) {
      if (copy_sync(c, hdr, dcomp + pos, nget, hipMemcpyDeviceToHost) != hipSuccess) return HBAM_EDEVICE;
    }
    if (avail == 0) return window_is_file_end ? HBAM_EEOF : HBAM_EMORE;
    const uint32_t blen = nget >= 18 ? (uint32_t)rd16(hdr + 16) + 1u : 0u;
    if (!window_is_file_end && (avail < 18 || blen > avail)) return HBAM_EMORE;
    if (avail >= 18 && blen >= 18 && blen <= avail && blen > 32) {
      // block header looks readable but was not accepted: classify with its footer
      std::vector<uint8_t> full(blen + 8);
      if (copy_sync(c, full.data(), dcomp + pos, blen, hipMemcpyDeviceToHost) != hipSuccess)
        return HBAM_EDEVICE;
      return readblock_error(full.data(), avail);
    }
    return readblock_error(hdr, avail);
  };
  if (first != start) {
    // the split's first block is not a BGZF block htsjdk accepts
    ch->nb = 0;
    ch->end_pos = start;
    ch->end_code = classify_end(start);
    return HBAM_OK;
  }
  if (bad == 0 || (bad == 1 && last.coff + last.clen > comp_len)) {
    // every link consistent (the last block may run past the window)
    uint64_t nb = ncand;
    if (last.coff + last.clen > comp_len) nb = ncand - 1;
    ch->nb = nb;
    ch->end_pos = (nb == ncand) ? last.coff + last.clen : last.coff;
    ch->end_code = classify_end(ch->end_pos);
    return HBAM_OK;
  }
  // slow path: walk the chain on the host over the candidate list
  std::vector<uint64_t> hc(ncand);
  std::vector<BlockRec> hb(ncand);
  HIPCHK(c, hipMemcpyAsync(hc.data(), cand, ncand * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(hb.data(), blk, ncand * sizeof(BlockRec), hipMemcpyDeviceToHost,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  std::vector<BlockRec> chain;
  uint64_t p = start;
  size_t idx = 0;
  for (;;) {
    auto it = std::lower_bound(hc.begin() + (long)idx, hc.end(), p);
    if (it == hc.end() || *it != p) break;
    idx = (size_t)(it - hc.begin());
    const BlockRec& r = hb[idx];
    if (r.coff + r.clen > comp_len || r.clen < 18) break;
    chain.push_back(r);
    p = r.coff + r.clen;
  }
  ch->nb = chain.size();
  ch->end_pos = p;
  ch->end_code = classify_end(p);
  HIPCHK(c, hipMemcpyAsync(blk, chain.data(), chain.size() * sizeof(BlockRec),
                           hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return HBAM_OK;
}

__global__ void k_isize32(const BlockRec* __restrict__ blk, uint64_t n, uint32_t* __restrict__ out,
                          uint32_t* __restrict__ big) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = blk[i].isize;
  out[i] = s <= 65536u ? s : 0u;
  if (s > 65536u) atomicMin(big, (uint32_t)i);
}

__global__ void k_first_bad_block(const int32_t* __restrict__ st, const uint32_t* __restrict__ crc,
                                  const BlockRec* __restrict__ blk, uint64_t n, int check_crc,
                                  unsigned long long* __restrict__ first) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool bad = st[i] != INF_OK;
  if (!bad && check_crc) bad = crc[i] != blk[i].crc;
  if (bad) atomicMin(first, (unsigned long long)i);
}

// empty BGZF blocks after the first (block order): flag[j] = 1 for an ISIZE-0 block
__global__ void k_empty_flags(const BlockRec* __restrict__ blk, uint64_t n, uint32_t* __restrict__ flag) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) flag[j] = (j >= 1 && blk[j].isize == 0) ? 1u : 0u;
}
__global__ void k_empty_scatter(const uint64_t* __restrict__ uoff, const uint32_t* __restrict__ flag,
                                const uint64_t* __restrict__ pos, uint64_t n, uint64_t* __restrict__ ev) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n && flag[j]) ev[pos[j]] = uoff[j];
}

int inflate_blocks(hbam_ctx* c, const uint8_t* dcomp, const BlockRec* blk, uint64_t nb,
                   const uint64_t* uoff, uint8_t* ubuf, int32_t* st, bool want_crc, uint32_t* crc) {
  uint8_t* lens;
  uint32_t *bitmap, *tails;
  uint8_t* edges;
  int rc;
  if ((rc = ensure(c, B_LENS, nb * LENS_SLOT, &lens))) return rc;
  if ((rc = ensure(c, B_BITMAP, nb * BITMAP_WORDS, &bitmap))) return rc;
  if ((rc = ensure(c, B_TAILS, 2 * nb + 2, &tails))) return rc;
  if ((rc = ensure(c, B_EDGE, 32 * nb + 32, &edges))) return rc;
  uint32_t* retry = nullptr;  // [MAX_SLICES counters][nb block indices]
  const bool wave = nb <= c->wave_max_blocks;
  if (wave) {
    if ((rc = ensure(c, B_RETRY, nb + MAX_SLICES, &retry))) return rc;
    HIPCHK(c, hipMemsetAsync(retry, 0, MAX_SLICES * 4, c->stream));
  }
  // Both passes are latency-bound at low occupancy (Huffman: 2 waves/SIMD; LZ77: a serial
  // walk per block), so the blocks are cut into slices and the LZ77 pass of slice s runs on a
  // second stream beside the Huffman pass of slice s+1: the CUs interleave the two kernels'
  // waves.  Slices share at most the 16-byte chunk at their boundary, whose bytes each side
  // writes bytewise (edge merge / LZ77 write-back), never the other side's.
  uint32_t ns = c->inflate_slices;
  if (ns < 1) ns = 1;
  if (ns > MAX_SLICES) ns = MAX_SLICES;
  if (!c->slices_forced && nb < (uint64_t)ns * 8192) ns = 1;  // small calls: one slice
  if (nb < ns) ns = 1;
  if (nb) {
    for (uint32_t si = 0; si < ns; ++si) {
      const uint64_t lo = nb * si / ns, hi = nb * (si + 1) / ns, n = hi - lo;
      if (!n) continue;
      hipStream_t rs = ns > 1 ? c->stream2 : c->stream;
      if (wave) {
        uint32_t* rl = retry + MAX_SLICES + lo;
        k_inflate_wave<<<(uint32_t)n, 64, 0, c->stream>>>(dcomp, blk + lo, uoff + lo, (uint32_t)n, ubuf,
                                                         bitmap + lo * BITMAP_WORDS, tails + 2 * lo,
                                                         edges + 32 * lo, st + lo, rl, retry + si);
        k_inflate_tokens<<<grid_for(n, INFLATE_WG), INFLATE_WG, 0, c->stream>>>(
            dcomp, blk + lo, uoff + lo, (uint32_t)n, ubuf, lens + lo * LENS_SLOT, bitmap + lo * BITMAP_WORDS,
            tails + 2 * lo, edges + 32 * lo, st + lo, rl, retry + si);
      } else {
        k_inflate_tokens<<<grid_for(n, INFLATE_WG), INFLATE_WG, 0, c->stream>>>(
            dcomp, blk + lo, uoff + lo, (uint32_t)n, ubuf, lens + lo * LENS_SLOT, bitmap + lo * BITMAP_WORDS,
            tails + 2 * lo, edges + 32 * lo, st + lo, nullptr, nullptr);
      }
      if (ns > 1) {
        HIPCHK(c, hipEventRecord(c->slice_ev[si], c->stream));
        HIPCHK(c, hipStreamWaitEvent(rs, c->slice_ev[si], 0));
      }
      if (si + 1 == ns) HIPCHK(c, hipEventRecord(c->ev[11], c->stream));
      k_edge_merge<<<grid_for(2 * n, 256), 256, 0, rs>>>(blk + lo, uoff + lo, (uint32_t)n, ubuf, edges + 32 * lo);
      k_resolve_units<<<(uint32_t)n, 64, 0, rs>>>(blk + lo, uoff + lo, (uint32_t)n, ubuf, bitmap + lo * BITMAP_WORDS,
                                                  tails + 2 * lo, st + lo);
    }
    if (ns > 1) {
      HIPCHK(c, hipEventRecord(c->slice_ev[MAX_SLICES], c->stream2));
      HIPCHK(c, hipStreamWaitEvent(c->stream, c->slice_ev[MAX_SLICES], 0));
    }
  }
  HIPCHK(c, hipGetLastError());
  if (wave && nb && getenv("HBAM_WV_STATS")) {  // diagnostics: blocks the wave pass left to the lane pass
    uint32_t cnt[MAX_SLICES];
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(cnt, retry, sizeof(cnt), hipMemcpyDeviceToHost));
    uint64_t tot = 0;
    for (uint32_t si = 0; si < MAX_SLICES; ++si) tot += cnt[si];
    fprintf(stderr, "hbam: wave inflate left %llu of %llu blocks to the lane pass\n", (unsigned long long)tot,
            (unsigned long long)nb);
#ifdef HBAM_WV_PROF
    unsigned long long pr[8];
    HIPCHK(c, hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_wvprof), sizeof(pr)));
    fprintf(stderr, "hbam: wave phases (Mcycles summed over waves): header %.1f tables %.1f count %.1f fix %.1f "
            "offsets %.1f write %.1f; fix rounds %llu over %llu DEFLATE blocks\n", pr[0] / 1e6, pr[1] / 1e6,
            pr[2] / 1e6, pr[3] / 1e6, pr[4] / 1e6, pr[5] / 1e6, pr[6], pr[7]);
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIPCHK(c, hipMemcpyToSymbol(HIP_SYMBOL(g_wvprof), z, sizeof(z)));
#endif
  }
  if (want_crc && nb) {
    k_crc32<<<grid_for(nb, 256), 256, 0, c->stream>>>(blk, uoff, (uint32_t)nb, ubuf, crc);
    HIPCHK(c, hipGetLastError());
  }
  return HBAM_OK;
}

}  // namespace

// =====================================================================================
extern "C" {

hbam_ctx* hbam_create(int device_ordinal, const hbam_opts* opts) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return nullptr;
  if (device_ordinal < 0 || device_ordinal >= ndev) return nullptr;
  if (hipSetDevice(device_ordinal) != hipSuccess) return nullptr;
  hbam_ctx* c = new hbam_ctx();
  c->device = device_ordinal;
  if (opts) c->opts = *opts;
  else c->opts.validate_refs = 1;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return nullptr;
  }
  if (hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess) {
    (void)hipStreamDestroy(c->stream);
    delete c;
    return nullptr;
  }
  for (auto& e : c->ev) (void)hipEventCreate(&e);
  for (auto& e : c->slice_ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  if (const char* sl = getenv("HBAM_INFLATE_SLICES")) {
    const long v = strtol(sl, nullptr, 10);
    if (v > 0) {
      c->inflate_slices = (uint32_t)v;
      c->slices_forced = true;
    }
  }
  if (const char* wm = getenv("HBAM_WAVE_MAX_BLOCKS")) c->wave_max_blocks = strtoull(wm, nullptr, 10);
  if (const char* gb = getenv("HBAM_GUESS_BATCH")) {
    const long v = strtol(gb, nullptr, 10);
    if (v > 0) c->guess_batch = (uint64_t)v;
  }
  if (hipHostMalloc((void**)&c->pinned_small, 4096, hipHostMallocDefault) != hipSuccess) {
    delete c;
    return nullptr;
  }
  return c;
}

void comm_detach(hbam_comm* m);  // hbam_comm.hip
void hbam_destroy(hbam_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  // a communicator that outlives its context keeps its device ordinal only (hbam_comm_destroy)
  for (hbam_comm* m : c->comms) comm_detach(m);
  for (auto& b : c->bufs)
    if (b.p) (void)hipFree(b.p);
  (void)hipStreamSynchronize(c->stream2);
  for (auto& e : c->ev) (void)hipEventDestroy(e);
  for (auto& e : c->slice_ev) (void)hipEventDestroy(e);
  if (c->pinned_small) (void)hipHostFree(c->pinned_small);
  if (c->rec_host) (void)hipHostFree(c->rec_host);
  (void)hipStreamDestroy(c->stream2);
  (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* hbam_last_error(const hbam_ctx* c) { return c ? c->err.c_str() : "null context"; }
void* hbam_stream(hbam_ctx* c) { return c ? (void*)c->stream : nullptr; }
int hbam_get_timing(const hbam_ctx* c, hbam_timing* out) {
  if (!c || !out) return HBAM_EINVAL;
  *out = c->timing;
  return HBAM_OK;
}

int hbam_upload(hbam_ctx* c, const uint8_t* host, uint64_t len, uint8_t** dev_out) {
  if (!c || !dev_out) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  uint8_t* d = nullptr;
  HIPCHK(c, hipMalloc(&d, len + 64));
  HIPCHK(c, hipMemsetAsync(d + len, 0, 64, c->stream));
  if (len) HIPCHK(c, hipMemcpyAsync(d, host, len, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  *dev_out = d;
  return HBAM_OK;
}

// Page-lock a caller-owned host range for this library's HIP runtime (hipHostRegister).  The
// streamed reader's host->device window copies are asynchronous only from page-locked memory;
// memory another runtime pinned (PyTorch-ROCm ships its own libamdhip64) is pageable here.
int hbam_host_register(hbam_ctx* c, void* host, uint64_t len) {
  if (!c || (len && !host)) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  if (!len) return HBAM_OK;
  const hipError_t e = hipHostRegister(host, len, hipHostRegisterDefault);
  if (e == hipErrorHostMemoryAlreadyRegistered) {
    (void)hipGetLastError();
    return HBAM_OK;
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_err(c, HBAM_EDEVICE, "hipHostRegister(%llu bytes): %s", (unsigned long long)len, hipGetErrorString(e));
  }
  return HBAM_OK;
}

int hbam_host_unregister(hbam_ctx* c, void* host) {
  if (!c || !host) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  const hipError_t e = hipHostUnregister(host);
  if (e != hipSuccess) (void)hipGetLastError();
  return HBAM_OK;
}

int hbam_download(hbam_ctx* c, const void* dev, uint64_t bytes, void* host) {
  if (!c || (bytes && (!dev || !host))) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, copy_sync(c, host, dev, bytes, hipMemcpyDeviceToHost));
  return HBAM_OK;
}

int hbam_device_free(hbam_ctx* c, uint8_t* dev) {
  if (!c) return HBAM_EINVAL;
  if (dev) HIPCHK(c, hipFree(dev));
  return HBAM_OK;
}

}  // extern "C"

namespace {

// Stage host bytes in the context's comp buffer (device, padded); return device ptr.
int stage_comp(hbam_ctx* c, const uint8_t* comp, int on_device, uint64_t len, const uint8_t** d) {
  if (on_device) {
    *d = comp;
    return HBAM_OK;
  }
  uint8_t* dc;
  int rc = ensure(c, B_COMP, len + 64, &dc);
  if (rc) return rc;
  HIPCHK(c, hipMemsetAsync(dc + len, 0, 64, c->stream));
  if (len) HIPCHK(c, hipMemcpyAsync(dc, comp, len, hipMemcpyHostToDevice, c->stream));
  *d = dc;
  return HBAM_OK;
}

// the @SQ lines of a SAM text header: SN value and LN, in order ([htsjdk] SAMTextHeaderCodec
// parseSQLine under the reader's STRICT stringency: an @SQ line without SN or LN, or an LN that is
// not an int, raises).  Returns false on such a line.
struct SqEntry {
  const uint8_t* name;
  uint32_t name_len;
  int32_t len;
};
bool text_sq_lines(const uint8_t* t, uint64_t n, std::vector<SqEntry>* out) {
  out->clear();
  for (uint64_t a = 0; a < n;) {
    uint64_t e = a;
    while (e < n && t[e] != '\n') ++e;
    uint64_t z = e;
    if (z > a && t[z - 1] == '\r') --z;  // "\r\n" ends a line too
    if (z - a >= 3 && t[a] == '@' && t[a + 1] == 'S' && t[a + 2] == 'Q' && (z - a == 3 || t[a + 3] == '\t')) {
      const uint8_t* sn = nullptr;
      uint32_t sn_len = 0;
      bool has_sn = false, has_ln = false;
      int64_t ln = 0;
      for (uint64_t f = a + 3; f < z;) {  // f at a '\t'
        uint64_t g = f + 1;
        while (g < z && t[g] != '\t') ++g;
        const uint8_t* v = t + f + 1;
        const uint64_t vl = g - f - 1;
        if (vl >= 3 && v[2] == ':' && v[0] == 'S' && v[1] == 'N' && !has_sn) {
          sn = v + 3;
          sn_len = (uint32_t)(vl - 3);
          has_sn = true;
        } else if (vl >= 3 && v[2] == ':' && v[0] == 'L' && v[1] == 'N' && !has_ln) {
          // Integer.parseInt: optional sign, then 1..10 digits within the int range
          uint64_t k = 3;
          bool neg = false;
          if (k < vl && (v[k] == '-' || v[k] == '+')) neg = v[k++] == '-';
          if (k == vl) return false;
          for (; k < vl; ++k) {
            if (v[k] < '0' || v[k] > '9') return false;
            ln = ln * 10 + (v[k] - '0');
            if (ln > 2147483648LL) return false;
          }
          if (neg) ln = -ln;
          if (ln > 2147483647LL) return false;
          has_ln = true;
        }
        f = g;
      }
      if (!has_sn || !has_ln) return false;
      out->push_back({sn, sn_len, (int32_t)ln});
    }
    a = e + 1;
  }
  return true;
}

// host-side BAM header parse over inflated bytes (SAMHeaderReader.readSAMHeaderFrom,
// SAMHeaderReader.java:53-72 -> [htsjdk] BAMFileReader.readHeader / readSequenceRecord): when the
// text holds @SQ lines, the binary dictionary must match it entry by entry — the count, each
// name (the binary name cut at its first whitespace, SAMSequenceUtil.truncateSequenceName) and
// each length — and every binary entry needs a name (l_name > 1); all SAMFormatException
int parse_header_bytes(const uint8_t* u, uint64_t n, hbam_header* h, bool* need_more) {
  *need_more = false;
  auto need = [&](uint64_t k) { return k > n; };
  if (need(8)) { *need_more = true; return HBAM_OK; }
  if (memcmp(u, "BAM\1", 4) != 0) return HBAM_EFORMAT;
  const int32_t l_text = rd32(u + 4);
  if (l_text < 0) return HBAM_EFORMAT;
  uint64_t p = 8 + (uint64_t)l_text;
  if (need(p + 4)) { *need_more = true; return HBAM_OK; }
  std::vector<SqEntry> sq;
  if (!text_sq_lines(u + 8, (uint64_t)l_text, &sq)) return HBAM_EFORMAT;
  const int32_t n_ref = rd32(u + p);
  if (n_ref < 0) return HBAM_EFORMAT;
  if (!sq.empty() && sq.size() != (size_t)n_ref) return HBAM_EFORMAT;
  p += 4;
  for (int32_t i = 0; i < n_ref; ++i) {
    if (need(p + 4)) { *need_more = true; return HBAM_OK; }
    const int32_t ln = rd32(u + p);
    if (ln <= 1) return HBAM_EFORMAT;  // "missing sequence name"
    if (need(p + 4 + (uint64_t)ln + 4)) { *need_more = true; return HBAM_OK; }
    if (!sq.empty()) {
      const uint8_t* nm = u + p + 4;
      uint32_t k = 0;
      while (k < (uint32_t)(ln - 1) && !(nm[k] == ' ' || (nm[k] >= 9 && nm[k] <= 13))) ++k;
      const SqEntry& t = sq[(size_t)i];
      if (t.name_len != k || memcmp(t.name, nm, k) != 0) return HBAM_EFORMAT;  // different names
      if (t.len != rd32(u + p + 4 + (uint64_t)ln)) return HBAM_EFORMAT;        // different lengths
    }
    p += 4 + (uint64_t)ln + 4;
  }
  h->l_text = l_text;
  h->n_ref = n_ref;
  h->header_ulen = p;
  return HBAM_OK;
}

}  // namespace

extern "C" {

int hbam_parse_header(hbam_ctx* c, const uint8_t* file, int on_device, uint64_t len,
                      hbam_header* out) {
  if (!c || !file || !out) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  const uint8_t* d;
  int rc = stage_comp(c, file, on_device, len, &d);
  if (rc) return rc;
  Chain ch;
  if ((rc = build_chain(c, d, len, 0, true, &ch))) return rc;
  if (ch.nb == 0) return set_err(c, ch.end_code == HBAM_EEOF ? HBAM_EFORMAT : ch.end_code,
                                 "no BGZF block at offset 0");
  // inflate a growing prefix of blocks until the header parses
  BlockRec* blk = (BlockRec*)c->bufs[B_BLK].p;
  uint64_t take = std::min<uint64_t>(ch.nb, 4);
  for (;;) {
    std::vector<BlockRec> hb(take);
    HIPCHK(c, copy_sync(c, hb.data(), blk, take * sizeof(BlockRec), hipMemcpyDeviceToHost));
    std::vector<uint64_t> uo(take + 1, 0);
    for (uint64_t i = 0; i < take; ++i) uo[i + 1] = uo[i] + std::min<uint32_t>(hb[i].isize, 65536u);
    uint64_t *duoff;
    uint8_t* ub;
    int32_t* st;
    if ((rc = ensure(c, B_UOFF, take + 1, &duoff))) return rc;
    if ((rc = ensure(c, B_UBUF, uo[take] + UBUF_SLACK, &ub))) return rc;
    if ((rc = ensure(c, B_INFST, take, &st))) return rc;
    HIPCHK(c, hipMemcpyAsync(duoff, uo.data(), (take + 1) * 8, hipMemcpyHostToDevice, c->stream));
    if ((rc = inflate_blocks(c, d, blk, take, duoff, ub, st, false, nullptr))) return rc;
    std::vector<int32_t> hst(take);
    std::vector<uint8_t> hu(uo[take] + 1);
    HIPCHK(c, hipMemcpyAsync(hst.data(), st, take * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(hu.data(), ub, uo[take], hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    uint64_t good = uo[take];
    for (uint64_t i = 0; i < take; ++i)
      if (hst[i] != INF_OK || hb[i].isize > 65536u) { good = uo[i]; break; }
    bool more = false;
    rc = parse_header_bytes(hu.data(), good, out, &more);
    if (rc) return set_err(c, rc, "invalid BAM header");
    if (!more) {
      // first voffset: normalized pointer after the header
      uint64_t p = out->header_ulen;
      uint64_t i = 0;
      while (i < take && uo[i + 1] <= p) ++i;
      if (i == take) {
        out->first_voffset = (hb[take - 1].coff + hb[take - 1].clen) << 16;
      } else {
        out->first_voffset = hb[i].coff << 16 | (p - uo[i]);
      }
      return HBAM_OK;
    }
    if (good < uo[take] || take == ch.nb)
      return set_err(c, HBAM_EFORMAT, "truncated BAM header");
    take = std::min<uint64_t>(ch.nb, take * 2);
  }
}

int hbam_scan_blocks(hbam_ctx* c, const uint8_t* comp, int on_device, uint64_t len,
                     uint64_t base_off, hbam_block* out, uint64_t cap, uint64_t* n_out) {
  if (!c || !comp || !n_out) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  const uint8_t* d;
  int rc = stage_comp(c, comp, on_device, len, &d);
  if (rc) return rc;
  Chain ch;
  if ((rc = build_chain(c, d, len, 0, true, &ch))) return rc;
  *n_out = ch.nb;
  if (out && ch.nb) {
    std::vector<BlockRec> hb(ch.nb);
    HIPCHK(c, copy_sync(c, hb.data(), c->bufs[B_BLK].p, ch.nb * sizeof(BlockRec),
                        hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < ch.nb && i < cap; ++i) {
      out[i].coff = hb[i].coff + base_off;
      out[i].clen = hb[i].clen;
      out[i].isize = hb[i].isize;
      out[i].crc = hb[i].crc;
      out[i].pad = 0;
    }
  }
  return ch.end_code == HBAM_EEOF ? HBAM_OK : set_err(c, ch.end_code, "BGZF chain ends at %llu",
                                                      (unsigned long long)ch.end_pos);
}

int hbam_inflate(hbam_ctx* c, const uint8_t* comp, int on_device, uint64_t comp_len,
                 const hbam_block* blks, uint64_t n, int check_crc, uint8_t* out, uint64_t out_cap,
                 uint64_t* out_off, int32_t* blk_status) {
  if (!c || !comp || (!blks && n)) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  const uint8_t* d;
  int rc = stage_comp(c, comp, on_device, comp_len, &d);
  if (rc) return rc;
  std::vector<BlockRec> hb(n);
  std::vector<uint64_t> uo(n + 1, 0);
  for (uint64_t i = 0; i < n; ++i) {
    if (blks[i].coff + blks[i].clen > comp_len || blks[i].clen < 18)
      return set_err(c, HBAM_EINVAL, "block %llu outside the buffer", (unsigned long long)i);
    hb[i].coff = blks[i].coff;
    hb[i].clen = blks[i].clen;
    hb[i].isize = blks[i].isize;
    hb[i].crc = blks[i].crc;
    hb[i].pad = 0;
    if (blks[i].isize > 65536u)
      return set_err(c, HBAM_EUNSUPPORTED, "ISIZE > 65536 in block %llu", (unsigned long long)i);
    uo[i + 1] = uo[i] + blks[i].isize;
  }
  if (out_off) memcpy(out_off, uo.data(), (n + 1) * 8);
  if (out && uo[n] > out_cap) return set_err(c, HBAM_EINVAL, "output buffer too small");
  BlockRec* db;
  uint64_t* duoff;
  uint8_t* ub;
  int32_t* st;
  uint32_t* crc;
  if ((rc = ensure(c, B_BLK, n + 1, &db))) return rc;
  if ((rc = ensure(c, B_UOFF, n + 1, &duoff))) return rc;
  if ((rc = ensure(c, B_UBUF, uo[n] + UBUF_SLACK, &ub))) return rc;
  if ((rc = ensure(c, B_INFST, n + 1, &st))) return rc;
  if ((rc = ensure(c, B_CRC, n + 1, &crc))) return rc;
  HIPCHK(c, hipMemcpyAsync(db, hb.data(), n * sizeof(BlockRec), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(duoff, uo.data(), (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
  if ((rc = inflate_blocks(c, d, db, n, duoff, ub, st, check_crc != 0, crc))) return rc;
  HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
  std::vector<int32_t> hst(n);
  std::vector<uint32_t> hcrc(n);
  HIPCHK(c, hipMemcpyAsync(hst.data(), st, n * 4, hipMemcpyDeviceToHost, c->stream));
  if (check_crc) HIPCHK(c, hipMemcpyAsync(hcrc.data(), crc, n * 4, hipMemcpyDeviceToHost, c->stream));
  if (out && uo[n]) HIPCHK(c, hipMemcpyAsync(out, ub, uo[n], hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[1]);
  c->timing = hbam_timing{};
  c->timing.inflate_ms = ms;
  c->timing.huffman_ms = ev_ms(c, 0, 11);
  c->timing.resolve_ms = ev_ms(c, 11, 1);
  c->timing.n_blocks = n;
  c->timing.ubuf_bytes = uo[n];
  for (uint64_t i = 0; i < n; ++i) {
    int32_t s = hst[i] == INF_OK ? HBAM_OK : hst[i] == INF_SHORT ? HBAM_EFORMAT : HBAM_EDATA;
    if (s == HBAM_OK && check_crc && hcrc[i] != hb[i].crc) s = HBAM_EFORMAT;
    if (blk_status) blk_status[i] = s;
  }
  return HBAM_OK;
}

}  // extern "C"

// =====================================================================================
// hbam_decode_split
// =====================================================================================
namespace {

int fill_columns(hbam_ctx* c, uint64_t n, DevColumns* dc) {
  int rc;
#define E(id, field, T)                                            \
  if ((rc = ensure(c, id, n + 1, (T**)&dc->field))) return rc;
  E(B_C_STATUS, status, int32_t)
  E(B_C_BS, block_size, int32_t)
  E(B_C_REF, ref_id, int32_t)
  E(B_C_POS, pos, int32_t)
  E(B_C_LRN, l_read_name, uint8_t)
  E(B_C_MAPQ, mapq, uint8_t)
  E(B_C_BIN, bin, uint16_t)
  E(B_C_NCIG, n_cigar, uint16_t)
  E(B_C_FLAG, flag, uint16_t)
  E(B_C_LSEQ, l_seq, int32_t)
  E(B_C_NREF, next_ref_id, int32_t)
  E(B_C_NPOS, next_pos, int32_t)
  E(B_C_TLEN, tlen, int32_t)
  E(B_C_KEY, key, int64_t)
  E(B_C_LAYOUT, layout_ok, uint8_t)
  E(B_C_NAMELEN, name_len, uint32_t)
  E(B_C_CIGN, cigar_n, uint32_t)
  E(B_C_SEQLEN, seq_len, uint32_t)
  E(B_C_AUXLEN, aux_len, uint32_t)
  E(B_C_NAMEOFF, name_off, uint64_t)
  E(B_C_CIGOFF, cigar_off, uint64_t)
  E(B_C_SEQOFF, seq_off, uint64_t)
  E(B_C_AUXOFF, aux_off, uint64_t)
#undef E
  return HBAM_OK;
}

float ev_ms(hbam_ctx* c, int a, int b) {
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev[a], c->ev[b]);
  return ms;
}

}  // namespace

extern "C" int hbam_decode_split(hbam_ctx* c, const uint8_t* comp, int on_device,
                                 uint64_t comp_base, uint64_t comp_len, uint64_t file_len,
                                 uint64_t v_start, uint64_t v_end, int32_t n_ref,
                                 hbam_columns* out) {
  if (!c || !comp || !out) return HBAM_EINVAL;
  memset(out, 0, sizeof *out);
  HIPCHK(c, hipSetDevice(c->device));
  c->timing = hbam_timing{};
  const uint8_t* d;
  int rc = stage_comp(c, comp, on_device, comp_len, &d);
  if (rc) return rc;
  if (n_ref < 0) {
    if (comp_base != 0) return set_err(c, HBAM_EINVAL, "n_ref < 0 needs the file start");
    hbam_header h;
    if ((rc = hbam_parse_header(c, d, 1, comp_len, &h))) {
      out->status = rc;
      return rc;
    }
    n_ref = h.n_ref;
  }
  const uint64_t coff_s = v_start >> 16;
  const uint32_t uoff_s = (uint32_t)(v_start & 0xffff);
  if (coff_s < comp_base || coff_s > comp_base + comp_len)
    return set_err(c, HBAM_EINVAL, "v_start outside the compressed window");
  const uint64_t start = coff_s - comp_base;
  const bool window_is_file_end = (comp_base + comp_len >= file_len);

  HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
  Chain ch;
  if ((rc = build_chain(c, d, comp_len, start, window_is_file_end, &ch))) return rc;
  HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
  BlockRec* blk = (BlockRec*)c->bufs[B_BLK].p;
  uint64_t nb = ch.nb;

  // ---- BCIS.seek(vStart): first block (empty -> the following one), offset checks
  if (nb == 0) {
    // readBlock at vStart's block fails (or EOF: count == 0 -> empty current block)
    if (ch.end_code == HBAM_EEOF) {
      // seek to a position at/after the end: empty block, offset must be 0 and eof
      if (uoff_s != 0) { out->status = HBAM_EIO; return HBAM_OK; }
      out->status = HBAM_OK;
      return HBAM_OK;
    }
    out->status = ch.end_code == HBAM_ERUNTIMEIO ? HBAM_EIO : ch.end_code;
    return HBAM_OK;
  }
  // blocks: table is device resident; ISIZE clamp + first oversized block
  uint32_t* isz;
  uint64_t* uoff;
  uint64_t* small;
  if ((rc = ensure(c, B_ISZ32, nb + 1, &isz))) return rc;
  if ((rc = ensure(c, B_UOFF, nb + 1, &uoff))) return rc;
  if ((rc = ensure(c, B_SMALL, 16, &small))) return rc;
  HIPCHK(c, hipMemsetAsync(small, 0xff, 8 * 8, c->stream));
  HIPCHK(c, hipMemsetAsync(small + 8, 0, 8 * 8, c->stream));
  k_isize32<<<grid_for(nb, 256), 256, 0, c->stream>>>(blk, nb, isz, (uint32_t*)small);
  if ((rc = scan_exclusive<uint32_t>(c, isz, nb, uoff, nullptr))) return rc;
  // the inflated total and the first blocks (host view, for the seek semantics): one round trip
  BlockRec b0[2];
  HIPCHK(c, hipMemcpyAsync(c->pinned_small + 64, uoff + nb, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->pinned_small + 66, blk, std::min<uint64_t>(nb, 2) * sizeof(BlockRec),
                           hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint64_t utotal = c->pinned_small[64];
  memcpy(b0, c->pinned_small + 66, std::min<uint64_t>(nb, 2) * sizeof(BlockRec));
  // inflate
  uint8_t* ub;
  int32_t* st;
  uint32_t* crc;
  if ((rc = ensure(c, B_UBUF, utotal + UBUF_SLACK, &ub))) return rc;
  if ((rc = ensure(c, B_INFST, nb + 1, &st))) return rc;
  if ((rc = ensure(c, B_CRC, nb + 1, &crc))) return rc;
  HIPCHK(c, hipEventRecord(c->ev[2], c->stream));
  if ((rc = inflate_blocks(c, d, blk, nb, uoff, ub, st, c->opts.check_crc != 0, crc))) return rc;
  HIPCHK(c, hipEventRecord(c->ev[3], c->stream));
  unsigned long long* first_bad = (unsigned long long*)small + 1;
  k_first_bad_block<<<grid_for(nb, 256), 256, 0, c->stream>>>(st, crc, blk, nb, c->opts.check_crc,
                                                             first_bad);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(c->pinned_small, small, 16, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  uint64_t fb = c->pinned_small[1];
  const uint32_t bigi = (uint32_t)(c->pinned_small[0] & 0xffffffffu);
  int32_t fb_code = HBAM_EEOF;
  if (fb != ~0ULL) {
    int32_t s;
    HIPCHK(c, copy_sync(c, &s, st + fb, 4, hipMemcpyDeviceToHost));
    fb_code = (s == INF_DATA) ? HBAM_EDATA : HBAM_EFORMAT;
  }
  if (bigi != 0xffffffffu && (fb == ~0ULL || bigi < fb)) {
    fb = bigi;
    fb_code = HBAM_EUNSUPPORTED;
  }
  // hard end: first failing block, else the chain end
  uint64_t hard_end;
  int32_t hard_code;
  if (fb != ~0ULL) {
    HIPCHK(c, copy_sync(c, &hard_end, uoff + fb, 8, hipMemcpyDeviceToHost));
    hard_code = fb_code;
  } else {
    hard_end = utotal;
    hard_code = ch.end_code;
  }
  // seek: block 0 (or 1 if block 0 is empty)
  uint64_t sblk = 0;
  if (b0[0].isize == 0) {
    if (fb == 0) { out->status = fb_code; return HBAM_OK; }
    sblk = 1;
  }
  if (fb == sblk) { out->status = fb_code; return HBAM_OK; }
  uint64_t r0;
  if (sblk >= nb) {
    // available() after an empty last block: EOF or readBlock error
    if (ch.end_code != HBAM_EEOF) { out->status = ch.end_code == HBAM_ERUNTIMEIO ? HBAM_EIO : ch.end_code; return HBAM_OK; }
    if (uoff_s != 0) { out->status = HBAM_EIO; return HBAM_OK; }
    out->status = HBAM_OK;
    return HBAM_OK;
  }
  {
    const BlockRec& bs = b0[sblk];
    const uint64_t after = comp_base + bs.coff + bs.clen;  // file position after the block
    const bool eof = (after == file_len) || (file_len - after == 28);
    if (uoff_s > bs.isize || (uoff_s == bs.isize && !eof)) { out->status = HBAM_EIO; return HBAM_OK; }
    // uoff[sblk] is 0: sblk is 1 only when block 0 is empty (uoff[1] = ISIZE 0)
    r0 = uoff_s;
  }
  // events: empty blocks after the seek block, at positions <= hard_end, in block order (so
  // sorted by position: k_decode_fixed binary-searches them; any number of them)
  uint64_t* evd;
  uint32_t* evflag;
  uint64_t* evpos;
  const uint64_t nbs = nb - sblk;
  if ((rc = ensure(c, B_EVFLAG, nbs + 1, &evflag)) || (rc = ensure(c, B_EVPOS, nbs + 1, &evpos))) return rc;
  k_empty_flags<<<grid_for(nbs, 256), 256, 0, c->stream>>>(blk + sblk, nbs, evflag);
  HIPCHK(c, hipGetLastError());
  // their count is read back with the record walk's stitch count below (one round trip); the
  // list is sized for every block
  if ((rc = scan_exclusive(c, evflag, nbs, evpos, nullptr))) return rc;
  if ((rc = ensure(c, B_EVENTS, nbs + 1, &evd))) return rc;
  k_empty_scatter<<<grid_for(nbs, 256), 256, 0, c->stream>>>(uoff + sblk, evflag, evpos, nbs, evd);
  HIPCHK(c, hipGetLastError());
  // events beyond the hard end cannot be reached; keep them (empty_at checks <= hard_end)

  // ---- K5: record starts (blocks [sblk, nb))
  const uint64_t wb = nb - sblk;
  const uint64_t* uo = uoff + sblk;
  uint64_t *entry, *exitp, *rbase, *rec_off, *voff;
  uint16_t* rel;
  uint32_t *count, *badlist;
  HIPCHK(c, hipEventRecord(c->ev[4], c->stream));
  if ((rc = ensure(c, B_ENTRY, wb + 1, &entry))) return rc;
  if ((rc = ensure(c, B_EXIT, wb + 1, &exitp))) return rc;
  if ((rc = ensure(c, B_REL, wb * WALK_CAP, &rel))) return rc;
  if ((rc = ensure(c, B_COUNT, wb + 1, &count))) return rc;
  if ((rc = ensure(c, B_RECBASE, wb + 1, &rbase))) return rc;
  if ((rc = ensure(c, B_BADLIST, wb + 1, &badlist))) return rc;
  if (wb > 1)
    k_block_entry<<<(uint32_t)(wb - 1), 64, 0, c->stream>>>(ub, uo, (uint32_t)wb, hard_end, BamFmt{n_ref},
                                                            entry);
  k_block_walk<<<grid_for(wb, 64), 64, 0, c->stream>>>(ub, uo, (uint32_t)wb, r0, hard_end, BamFmt{n_ref},
                                                       entry, rel, count, exitp);
  uint32_t* nbad_d = (uint32_t*)(small + 5);
  uint8_t* mark;
  if ((rc = ensure(c, B_MARK, wb + 1, &mark))) return rc;
  HIPCHK(c, hipMemsetAsync(nbad_d, 0, 4, c->stream));
  HIPCHK(c, hipMemsetAsync(mark, 0, 1, c->stream));  // block 0 (the split start) is never listed
  if (wb > 1)
    k_stitch_check<<<grid_for(wb - 1, 256), 256, 0, c->stream>>>(entry, exitp, (uint32_t)wb, nbad_d,
                                                                 badlist, (uint32_t)wb, mark);
  HIPCHK(c, hipMemcpyAsync(c->pinned_small + 80, nbad_d, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->pinned_small + 81, evpos + nbs, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  uint32_t nbad = (uint32_t)c->pinned_small[80];
  const uint64_t nev64 = c->pinned_small[81];
  if (nev64 > 0xffffffffull) return set_err(c, HBAM_EUNSUPPORTED, "more than 2^32-1 empty BGZF blocks");
  const uint32_t nev = (uint32_t)nev64;
  if (nbad) {  // runs of mismatched blocks repaired in parallel, then whatever is left, in order
    k_chain_fix_par<<<grid_for(nbad, 64), 64, 0, c->stream>>>(ub, uo, (uint32_t)wb, hard_end, BamFmt{n_ref},
                                                               entry, rel, count, exitp, badlist, nbad, mark);
    HIPCHK(c, hipMemsetAsync(nbad_d, 0, 4, c->stream));
    k_stitch_check<<<grid_for(wb - 1, 256), 256, 0, c->stream>>>(entry, exitp, (uint32_t)wb, nbad_d,
                                                                 badlist, (uint32_t)wb, nullptr);
    HIPCHK(c, hipMemcpyAsync(&nbad, nbad_d, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  if (nbad) {
    // sort the mismatch list (atomic order is arbitrary)
    std::vector<uint32_t> bl(nbad);
    HIPCHK(c, copy_sync(c, bl.data(), badlist, nbad * 4, hipMemcpyDeviceToHost));
    std::sort(bl.begin(), bl.end());
    HIPCHK(c, copy_sync(c, badlist, bl.data(), nbad * 4, hipMemcpyHostToDevice));
    k_chain_fix<<<1, 64, 0, c->stream>>>(ub, uo, (uint32_t)wb, hard_end, BamFmt{n_ref}, entry, rel, count,
                                         exitp, badlist, nbad);
    HIPCHK(c, hipGetLastError());
  }
  uint64_t nrec = 0;
  if ((rc = scan_exclusive<uint32_t>(c, count, wb, rbase, &nrec))) return rc;
  if ((rc = ensure(c, B_RECOFF, nrec + 1, &rec_off))) return rc;
  if ((rc = ensure(c, B_VOFF, nrec + 1, &voff))) return rc;
  k_emit_offsets<<<(uint32_t)wb, 256, 0, c->stream>>>(uo, blk + sblk, (uint32_t)wb, rel, count, rbase,
                                                      comp_base, rec_off, voff);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->ev[5], c->stream));

  // ---- K6/K7/K8
  DevColumns dc{};
  if ((rc = fill_columns(c, nrec, &dc))) return rc;
  unsigned long long* first_stop = (unsigned long long*)small + 6;
  HIPCHK(c, hipMemsetAsync(first_stop, 0xff, 8, c->stream));
  if (nrec)
    k_decode_fixed<<<grid_for(nrec, 256), 256, 0, c->stream>>>(
        ub, nrec, rec_off, voff, v_end, hard_end, hard_code, evd, nev, n_ref, c->opts.validate_refs,
        dc, first_stop);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->ev[6], c->stream));
  uint64_t fs;
  HIPCHK(c, hipMemcpyAsync(&fs, first_stop, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  uint64_t n_final = std::min<uint64_t>(fs, nrec);
  int32_t status = HBAM_OK;
  uint64_t err_rec = 0;
  if (fs < nrec) {
    int32_t s;
    HIPCHK(c, copy_sync(c, &s, dc.status + fs, 4, hipMemcpyDeviceToHost));
    if (s < 0) {
      status = s;
      err_rec = fs;
    }
  } else if (hard_code == HBAM_EMORE) {
    // The window ends exactly at a record boundary.  Withhold the last record so that the next
    // window re-reads it together with what follows: that is where the reference's read()
    // meets an empty BGZF block at the boundary (which ends the split).
    n_final = nrec ? nrec - 1 : 0;
    status = HBAM_EMORE;
    err_rec = n_final;
  }
  if (status == HBAM_EMORE) {
    // resume point for the next window: the stop record's voffset (already in voff[n_final]
    // when that record was walked), else v_start
    if (n_final >= nrec) HIPCHK(c, copy_sync(c, voff + n_final, &v_start, 8, hipMemcpyHostToDevice));
  }
  // ---- pools
  uint64_t tot_name = 0, tot_cig = 0, tot_seq = 0, tot_aux = 0;
  // the four pool scans in one pass (k_scan4_*), their totals read back in one round trip
  {
    const uint32_t tiles = (uint32_t)std::max<uint64_t>(1, (n_final + SCAN4_TILE - 1) / SCAN4_TILE);
    uint64_t* partial;
    if ((rc = ensure(c, B_PARTIAL, 4ull * tiles + 1, &partial))) return rc;
    const Scan4In in{{dc.name_len, dc.cigar_n, dc.seq_len, dc.aux_len}};
    const Scan4Out so{{dc.name_off, dc.cigar_off, dc.seq_off, dc.aux_off}};
    k_scan4_reduce<<<tiles, 256, 0, c->stream>>>(in, n_final, partial, tiles);
    k_scan4_partials<<<4, 256, 0, c->stream>>>(partial, tiles, so, n_final);
    k_scan4_apply<<<tiles, 256, 0, c->stream>>>(in, n_final, partial, tiles, so);
    HIPCHK(c, hipGetLastError());
  }
  {
    const uint64_t* offs[4] = {dc.name_off, dc.cigar_off, dc.seq_off, dc.aux_off};
    for (int q = 0; q < 4; ++q)
      HIPCHK(c, hipMemcpyAsync(c->pinned_small + 96 + q, offs[q] + n_final, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    tot_name = c->pinned_small[96];
    tot_cig = c->pinned_small[97];
    tot_seq = c->pinned_small[98];
    tot_aux = c->pinned_small[99];
  }
  if ((rc = ensure(c, B_C_NAMES, tot_name + 1, &dc.names))) return rc;
  if ((rc = ensure(c, B_C_CIGARS, tot_cig + 1, &dc.cigars))) return rc;
  if ((rc = ensure(c, B_C_SEQ, tot_seq + 1, &dc.seq))) return rc;
  if ((rc = ensure(c, B_C_QUAL, tot_seq + 1, &dc.qual))) return rc;
  if ((rc = ensure(c, B_C_AUX, tot_aux + 1, &dc.aux))) return rc;
  HIPCHK(c, hipEventRecord(c->ev[7], c->stream));
  if (n_final)
    k_decode_pools<<<(uint32_t)std::min<uint64_t>(grid_for(n_final, 256), POOLS_MAX_WG), 256, 0, c->stream>>>(
        ub, n_final, rec_off, dc);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->ev[8], c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));

  out->n_records = n_final;
  out->status = status;
  out->err_record = err_rec;
  out->voffset = voff;
  out->key = dc.key;
  out->rec_off = rec_off;
  out->ubuf = ub;
  out->ubuf_len = utotal;
  out->block_size = dc.block_size;
  out->ref_id = dc.ref_id;
  out->pos = dc.pos;
  out->l_read_name = dc.l_read_name;
  out->mapq = dc.mapq;
  out->bin = dc.bin;
  out->n_cigar = dc.n_cigar;
  out->flag = dc.flag;
  out->l_seq = dc.l_seq;
  out->next_ref_id = dc.next_ref_id;
  out->next_pos = dc.next_pos;
  out->tlen = dc.tlen;
  out->layout_ok = dc.layout_ok;
  out->name_off = dc.name_off;
  out->names = dc.names;
  out->cigar_off = dc.cigar_off;
  out->cigars = dc.cigars;
  out->seq_off = dc.seq_off;
  out->seq = dc.seq;
  out->qual = dc.qual;
  out->aux_off = dc.aux_off;
  out->aux = dc.aux;

  c->timing.scan_ms = ev_ms(c, 0, 1);
  c->timing.inflate_ms = ev_ms(c, 2, 3);
  c->timing.huffman_ms = ev_ms(c, 2, 11);
  c->timing.resolve_ms = ev_ms(c, 11, 3);
  c->timing.walk_ms = ev_ms(c, 4, 5);
  c->timing.decode_ms = ev_ms(c, 5, 6);
  c->timing.pools_ms = ev_ms(c, 7, 8);
  c->timing.total_ms = ev_ms(c, 0, 8);
  c->timing.n_blocks = nb;
  c->timing.comp_bytes = ch.end_pos - start;
  c->timing.ubuf_bytes = utotal;
  c->timing.n_records = n_final;
  c->timing.pool_bytes = tot_name + 4 * tot_cig + 2 * tot_seq + tot_aux;
  return HBAM_OK;
}

// ---- streamed split read over host-resident file bytes (config #4) -------------------------
struct hbam_split_stream {
  hbam_ctx* c = nullptr;
  const uint8_t* file = nullptr;
  uint64_t file_len = 0, v_cur = 0, v_end = 0, win = 0;
  uint64_t limit = 0;  // no window reaches past this file offset (split-local reads, see split_limit)
  int32_t n_ref = 0;
  // read-callback streams (hbam_split_open_reader): pinned host staging per window slot
  hbam_read_fn read = nullptr;
  void* user = nullptr;
  uint8_t* hbuf[2] = {nullptr, nullptr};
  uint64_t hcap[2] = {0, 0};
  uint64_t hbase[2] = {0, 0}, hlen[2] = {0, 0};  // file bytes each staging slot holds
  uint64_t read_bytes = 0;  // bytes requested from the callback
  uint8_t* dbuf[2] = {nullptr, nullptr};
  uint64_t dcap[2] = {0, 0};
  uint64_t base[2] = {0, 0}, len[2] = {0, 0};
  bool valid[2] = {false, false}, pending[2] = {false, false};
  hipStream_t cs = nullptr;
  hipEvent_t e0[2] = {nullptr, nullptr}, e1[2] = {nullptr, nullptr};
  bool done = false;
  uint64_t h2d_bytes = 0, windows = 0;
  double h2d_ms = 0;
  uint8_t* rec_host = nullptr;  // hbam_split_records_to_host: pinned, grow-only
  size_t rec_host_cap = 0;
};

namespace {
constexpr uint64_t STREAM_OVERLAP = 256 << 10;  // predicted resume point: within the last 256 KiB

int stream_wait(hbam_split_stream* s, int k) {
  if (!s->pending[k]) return HBAM_OK;
  hbam_ctx* c = s->c;
  HIPCHK(c, hipEventSynchronize(s->e1[k]));
  float ms = 0;
  (void)hipEventElapsedTime(&ms, s->e0[k], s->e1[k]);
  s->h2d_ms += ms;
  s->h2d_bytes += s->len[k];
  s->pending[k] = false;
  return HBAM_OK;
}

// Split-local bound: a FileVirtualSplit [v_start, v_end) reads records starting before v_end,
// i.e. in blocks at coff <= v_end >> 16; the last of them may run into the next blocks, and the
// reader stops at the first record at or after v_end, which starts in a block that begins within
// 64 KiB after that.  Windows never reach past (v_end >> 16) + SPLIT_TAIL; when a window so cut
// holds no complete record (a record longer than the tail) the bound moves out (hbam_split_next).
constexpr uint64_t SPLIT_TAIL = 3ull << 16;
uint64_t split_limit(uint64_t v_end, uint64_t file_len) {
  const uint64_t e = v_end >> 16;
  return e >= file_len || file_len - e <= SPLIT_TAIL ? file_len : e + SPLIT_TAIL;
}

// read-callback streams: file bytes [b, b + n) into host staging slot k.  Whatever either slot's
// staging already holds (the windows' overlap, a window re-copied at a resume point) is copied
// from there — slot k's own bytes first, by one memmove, before anything else lands in its
// buffer — and only the rest is asked of the callback, so every file byte is read once.
int stream_stage(hbam_split_stream* s, int k, uint64_t b, uint64_t n) {
  hbam_ctx* c = s->c;
  const uint64_t e = b + n;
  uint8_t* dst = s->hbuf[k];
  uint8_t* fresh = nullptr;
  if (s->hcap[k] < n + 64) {
    if (hipHostMalloc((void**)&fresh, n + 64, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      return set_err(c, HBAM_ENOMEM, "hbam_split_next: hipHostMalloc(%llu) failed", (unsigned long long)(n + 64));
    }
    dst = fresh;
  }
  // covered[] = the new range's bytes already in place, as [lo, hi) file intervals
  uint64_t cov_lo[2] = {0, 0}, cov_hi[2] = {0, 0};
  int ncov = 0;
  auto take = [&](int src) {
    if (!s->hbuf[src] || !s->hlen[src]) return;
    const uint64_t lo = std::max(b, s->hbase[src]), hi = std::min(e, s->hbase[src] + s->hlen[src]);
    if (lo >= hi) return;
    memmove(dst + (lo - b), s->hbuf[src] + (lo - s->hbase[src]), hi - lo);
    cov_lo[ncov] = lo;
    cov_hi[ncov] = hi;
    ++ncov;
  };
  take(k);  // own bytes first (in place: a single memmove)
  // the other slot's, outside what slot k supplied
  if (s->hbuf[1 - k] && s->hlen[1 - k]) {
    const int o = 1 - k;
    uint64_t lo = std::max(b, s->hbase[o]), hi = std::min(e, s->hbase[o] + s->hlen[o]);
    if (ncov && lo < hi) {  // clip to the part not covered yet (k's cover is one interval)
      if (lo >= cov_lo[0] && hi <= cov_hi[0]) lo = hi;
      else if (lo >= cov_lo[0] && lo < cov_hi[0]) lo = cov_hi[0];
      else if (hi > cov_lo[0] && hi <= cov_hi[0]) hi = cov_lo[0];
    }
    if (lo < hi) {
      memcpy(dst + (lo - b), s->hbuf[o] + (lo - s->hbase[o]), hi - lo);
      cov_lo[ncov] = lo;
      cov_hi[ncov] = hi;
      ++ncov;
    }
  }
  // the gaps, from the callback
  uint64_t p = b;
  while (p < e) {
    bool moved = false;
    for (int q = 0; q < ncov; ++q)
      if (p >= cov_lo[q] && p < cov_hi[q]) {
        p = cov_hi[q];
        moved = true;
      }
    if (moved) continue;
    uint64_t stop = e;
    for (int q = 0; q < ncov; ++q)
      if (cov_lo[q] > p) stop = std::min(stop, cov_lo[q]);
    while (p < stop) {
      const int64_t got = s->read(s->user, p, stop - p, dst + (p - b));
      if (got <= 0) {
        if (fresh) (void)hipHostFree(fresh);
        return set_err(c, HBAM_EIO, "hbam_split_next: read(%llu, %llu) returned %lld", (unsigned long long)p,
                       (unsigned long long)(stop - p), (long long)got);
      }
      s->read_bytes += std::min<uint64_t>((uint64_t)got, stop - p);
      p += std::min<uint64_t>((uint64_t)got, stop - p);
    }
  }
  if (fresh) {
    if (s->hbuf[k]) HIPCHK(c, hipHostFree(s->hbuf[k]));
    s->hbuf[k] = fresh;
    s->hcap[k] = n + 64;
  }
  s->hbase[k] = b;
  s->hlen[k] = n;
  return HBAM_OK;
}

// copy file bytes [b, b + n) into window buffer k on the copy stream (asynchronous)
int stream_copy(hbam_split_stream* s, int k, uint64_t b, uint64_t n) {
  hbam_ctx* c = s->c;
  int rc = stream_wait(s, k);
  if (rc) return rc;
  if (s->read && n && (rc = stream_stage(s, k, b, n))) return rc;
  if (s->dcap[k] < n + 64) {
    if (s->dbuf[k]) HIPCHK(c, hipFree(s->dbuf[k]));
    s->dbuf[k] = nullptr;
    s->dcap[k] = 0;
    if (hipMalloc(&s->dbuf[k], n + 64) != hipSuccess) {
      (void)hipGetLastError();
      return set_err(c, HBAM_ENOMEM, "hbam_split_next: hipMalloc(%llu) failed", (unsigned long long)(n + 64));
    }
    s->dcap[k] = n + 64;
  }
  HIPCHK(c, hipEventRecord(s->e0[k], s->cs));
  if (n) HIPCHK(c, hipMemcpyAsync(s->dbuf[k], s->read ? s->hbuf[k] : s->file + b, n, hipMemcpyHostToDevice, s->cs));
  HIPCHK(c, hipMemsetAsync(s->dbuf[k] + n, 0, 64, s->cs));
  HIPCHK(c, hipEventRecord(s->e1[k], s->cs));
  s->base[k] = b;
  s->len[k] = n;
  s->valid[k] = true;
  s->pending[k] = true;
  return HBAM_OK;
}
}  // namespace

namespace {
hbam_split_stream* split_open(hbam_ctx* c, const uint8_t* file, hbam_read_fn read, void* user,
                              uint64_t file_len, uint64_t v_start, uint64_t v_end, int32_t n_ref,
                              uint64_t window_bytes) {
  if (!c || n_ref < 0) return nullptr;
  if (hipSetDevice(c->device) != hipSuccess) return nullptr;
  hbam_split_stream* s = new hbam_split_stream();
  s->c = c;
  s->file = file;
  s->read = read;
  s->user = user;
  s->file_len = file_len;
  s->v_cur = v_start;
  s->v_end = v_end;
  s->limit = split_limit(v_end, file_len);
  s->n_ref = n_ref;
  s->win = std::max<uint64_t>(window_bytes, 1 << 16);
  bool ok = hipStreamCreateWithFlags(&s->cs, hipStreamNonBlocking) == hipSuccess;
  for (int k = 0; k < 2 && ok; ++k)
    ok = hipEventCreate(&s->e0[k]) == hipSuccess && hipEventCreate(&s->e1[k]) == hipSuccess;
  if (!ok) {
    (void)hipGetLastError();
    hbam_split_close(s);
    return nullptr;
  }
  return s;
}
}  // namespace

extern "C" hbam_split_stream* hbam_split_open(hbam_ctx* c, const uint8_t* file, uint64_t file_len,
                                         uint64_t v_start, uint64_t v_end, int32_t n_ref,
                                         uint64_t window_bytes) {
  if (!file && file_len) return nullptr;
  return split_open(c, file, nullptr, nullptr, file_len, v_start, v_end, n_ref, window_bytes);
}

extern "C" hbam_split_stream* hbam_split_open_reader(hbam_ctx* c, hbam_read_fn read, void* user,
                                                     uint64_t file_len, uint64_t v_start, uint64_t v_end,
                                                     int32_t n_ref, uint64_t window_bytes) {
  if (!read) return nullptr;
  return split_open(c, nullptr, read, user, file_len, v_start, v_end, n_ref, window_bytes);
}

extern "C" int hbam_split_next(hbam_split_stream* s, hbam_columns* out) {
  if (!s || !out) return HBAM_EINVAL;
  hbam_ctx* c = s->c;
  memset(out, 0, sizeof *out);
  if (s->done) return 0;
  HIPCHK(c, hipSetDevice(c->device));
  for (;;) {
    const uint64_t ws = std::min(s->v_cur >> 16, s->file_len);
    const uint64_t lim = std::max(s->limit, ws);
    const uint64_t ahead = std::min<uint64_t>(s->win / 2, lim - ws);
    int k = -1;
    for (int b = 0; b < 2; ++b)
      if (s->valid[b] && s->base[b] <= ws && s->base[b] + s->len[b] >= ws + ahead &&
          (ws < s->base[b] + s->len[b] || s->base[b] + s->len[b] == lim))
        k = b;
    if (k < 0) {  // not predicted (first window, long record, grown window): copy it now
      k = s->valid[0] && !s->valid[1] ? 1 : 0;
      int rc = stream_copy(s, k, ws, std::min(s->win, lim - ws));
      if (rc) return rc;
    }
    int rc = stream_wait(s, k);
    if (rc) return rc;
    // prefetch the predicted next window into the other buffer while this one decodes
    const uint64_t wend = s->base[k] + s->len[k];
    const int o = 1 - k;
    if (wend < lim) {
      const uint64_t ov = std::min<uint64_t>(STREAM_OVERLAP, s->win / 2);
      const uint64_t ps = std::max(s->base[k], wend > ov ? wend - ov : 0);
      if (!(s->valid[o] && s->base[o] == ps))
        if ((rc = stream_copy(s, o, ps, std::min(s->win, lim - ps)))) return rc;
    }
    ++s->windows;
    const uint8_t* w = s->dbuf[k] ? s->dbuf[k] : (const uint8_t*)s->dbuf[o];
    if (!w) {  // empty file: nothing was ever allocated
      if ((rc = stream_copy(s, k, ws, 0)) || (rc = stream_wait(s, k))) return rc;
      w = s->dbuf[k];
    }
    rc = hbam_decode_split(c, w, 1, s->base[k], s->len[k], s->file_len, s->v_cur, s->v_end, s->n_ref, out);
    if (rc) return rc;
    if (out->status != HBAM_EMORE) {
      s->done = true;
      return 1;
    }
    uint64_t resume = s->v_cur;
    if (out->voffset) HIPCHK(c, copy_sync(c, &resume, out->voffset + out->n_records, 8, hipMemcpyDeviceToHost));
    out->status = HBAM_OK;
    out->err_record = 0;
    if (resume == s->v_cur && out->n_records == 0) {
      // not one record fits: a longer window, copied at the resume point (past the split-local
      // bound too when the window was cut there)
      if (wend >= s->file_len)
        return set_err(c, HBAM_EINVAL, "hbam_split_next: no progress at voffset %llu", (unsigned long long)s->v_cur);
      for (int b = 0; b < 2; ++b) {
        if ((rc = stream_wait(s, b))) return rc;
        s->valid[b] = false;
      }
      if (wend >= lim) s->limit = std::min(s->file_len, lim + std::max<uint64_t>(s->win, SPLIT_TAIL));
      else s->win *= 2;
      continue;
    }
    s->v_cur = resume;
    if (out->n_records) return 1;
  }
}

extern "C" int hbam_split_stats(const hbam_split_stream* s, uint64_t* h2d_bytes, double* h2d_ms, uint64_t* windows) {
  if (!s) return HBAM_EINVAL;
  if (h2d_bytes) *h2d_bytes = s->h2d_bytes;
  if (h2d_ms) *h2d_ms = s->h2d_ms;
  if (windows) *windows = s->windows;
  return HBAM_OK;
}

extern "C" uint64_t hbam_split_read_bytes(const hbam_split_stream* s) { return s ? s->read_bytes : 0; }

extern "C" void hbam_split_close(hbam_split_stream* s) {
  if (!s) return;
  (void)hipSetDevice(s->c->device);
  if (s->cs) (void)hipStreamSynchronize(s->cs);
  for (int k = 0; k < 2; ++k) {
    if (s->dbuf[k]) (void)hipFree(s->dbuf[k]);
    if (s->hbuf[k]) (void)hipHostFree(s->hbuf[k]);
    if (s->e0[k]) (void)hipEventDestroy(s->e0[k]);
    if (s->e1[k]) (void)hipEventDestroy(s->e1[k]);
  }
  if (s->cs) (void)hipStreamDestroy(s->cs);
  if (s->rec_host) (void)hipHostFree(s->rec_host);
  delete s;
}

extern "C" void hbam_free_host_columns(hbam_columns* h);
namespace {
int columns_to_host_impl(hbam_ctx* c, const hbam_columns* dv, hbam_columns* h) {
  const uint64_t n = dv->n_records;
  h->n_records = n;
  h->status = dv->status;
  h->err_record = dv->err_record;
  h->ubuf_len = dv->ubuf_len;
  auto cp = [&](void* dst, const void* src, size_t bytes) -> int {
    if (!bytes) return HBAM_OK;
    if (!src) return HBAM_EINVAL;
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    return HBAM_OK;
  };
#define ALLOC(field, T, cnt)                                          \
  h->field = (T*)malloc(sizeof(T) * ((cnt) ? (cnt) : 1));              \
  if (!h->field) return HBAM_ENOMEM;                                  \
  if ((rc = cp(h->field, dv->field, sizeof(T) * (cnt)))) return rc;
  int rc;
  ALLOC(voffset, uint64_t, n)
  ALLOC(key, int64_t, n)
  ALLOC(rec_off, uint64_t, n)
  ALLOC(block_size, int32_t, n)
  ALLOC(ref_id, int32_t, n)
  ALLOC(pos, int32_t, n)
  ALLOC(l_read_name, uint8_t, n)
  ALLOC(mapq, uint8_t, n)
  ALLOC(bin, uint16_t, n)
  ALLOC(n_cigar, uint16_t, n)
  ALLOC(flag, uint16_t, n)
  ALLOC(l_seq, int32_t, n)
  ALLOC(next_ref_id, int32_t, n)
  ALLOC(next_pos, int32_t, n)
  ALLOC(tlen, int32_t, n)
  ALLOC(layout_ok, uint8_t, n)
  ALLOC(name_off, uint64_t, n + 1)
  ALLOC(cigar_off, uint64_t, n + 1)
  ALLOC(seq_off, uint64_t, n + 1)
  ALLOC(aux_off, uint64_t, n + 1)
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint64_t nn = n ? h->name_off[n] : 0, nc = n ? h->cigar_off[n] : 0,
                 ns = n ? h->seq_off[n] : 0, na = n ? h->aux_off[n] : 0;
  ALLOC(names, uint8_t, nn)
  ALLOC(cigars, uint32_t, nc)
  ALLOC(seq, uint8_t, ns)
  ALLOC(qual, uint8_t, ns)
  ALLOC(aux, uint8_t, na)
  // the records' bytes (SAMRecordWritable payloads: block_size + record), rec_off rebased to them
  uint64_t lo = 0, hi = 0;
  if (n) {
    lo = h->rec_off[0];
    hi = h->rec_off[n - 1] + 4 + (uint64_t)(uint32_t)h->block_size[n - 1];
    if (hi < lo || hi > dv->ubuf_len + UBUF_SLACK)
      return set_err(c, HBAM_EINVAL, "hbam_columns_to_host: record bytes outside ubuf");
  }
  h->ubuf = (uint8_t*)malloc(hi > lo ? hi - lo : 1);
  if (!h->ubuf) return HBAM_ENOMEM;
  if ((rc = cp(h->ubuf, dv->ubuf + lo, hi - lo))) return rc;
#undef ALLOC
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (uint64_t i = 0; i < n; ++i) h->rec_off[i] -= lo;
  h->ubuf_len = hi - lo;
  return HBAM_OK;
}
}  // namespace

extern "C" int hbam_columns_to_host(hbam_ctx* c, const hbam_columns* dv, hbam_columns* h) {
  if (!c || !dv || !h) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  memset(h, 0, sizeof *h);
  const int rc = columns_to_host_impl(c, dv, h);
  if (rc != HBAM_OK) {
    // every error return leaves no host arrays behind; the copies already queued
    // into them must land before they are freed
    (void)hipStreamSynchronize(c->stream);
    hbam_free_host_columns(h);
  }
  return rc;
}

extern "C" void hbam_free_host_columns(hbam_columns* h) {
  if (!h) return;
  void* ps[] = {h->voffset, h->key, h->rec_off, h->block_size, h->ref_id, h->pos, h->l_read_name,
                h->mapq, h->bin, h->n_cigar, h->flag, h->l_seq, h->next_ref_id, h->next_pos, h->tlen,
                h->layout_ok, h->name_off, h->cigar_off, h->seq_off, h->aux_off, h->names, h->cigars,
                h->seq, h->qual, h->aux, h->ubuf};
  for (void* p : ps) free(p);
  memset(h, 0, sizeof *h);
}

namespace {
// rec_off rebased to the copied byte range; a record that does not end where the next one starts
// (columns that are not a decoded split's contiguous, ascending records) raises *bad
__global__ void k_rebase_off(const uint64_t* __restrict__ in, const int32_t* __restrict__ bs, uint64_t n,
                             uint64_t lo, uint64_t* __restrict__ out, uint32_t* __restrict__ bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = in[i];
    out[i] = r - lo;
    if (i + 1 < n && in[i + 1] != r + 4u + (uint64_t)(uint32_t)bs[i]) *bad = 1u;
  }
}

// Records-only host copy (hbam_records_to_host / hbam_split_records_to_host) into the pinned
// staging *stage (grow-only, *cap bytes)
int records_to_host(hbam_ctx* c, const hbam_columns* dv, hbam_columns* h, uint8_t** stage, size_t* cap) {
  HIPCHK(c, hipSetDevice(c->device));
  memset(h, 0, sizeof *h);
  const uint64_t n = dv->n_records;
  h->n_records = n;
  h->status = dv->status;
  h->err_record = dv->err_record;
  if (!n) return HBAM_OK;
  if (!dv->voffset || !dv->key || !dv->rec_off || !dv->block_size || !dv->ubuf) return HBAM_EINVAL;
  // the records' byte range: first record's offset .. last record's end
  HIPCHK(c, hipMemcpyAsync(c->pinned_small, dv->rec_off, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->pinned_small + 1, dv->rec_off + (n - 1), 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->pinned_small + 2, dv->block_size + (n - 1), 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint64_t lo = c->pinned_small[0];
  const uint64_t hi = c->pinned_small[1] + 4 + (uint64_t)(uint32_t)c->pinned_small[2];
  if (hi < lo || hi > dv->ubuf_len + UBUF_SLACK)
    return set_err(c, HBAM_EINVAL, "hbam_records_to_host: record bytes outside ubuf");
  const size_t cols = 8 * n * 3 + ((4 * n + 7) & ~(size_t)7);
  const size_t need = cols + (hi - lo) + 64;
  if (*cap < need) {
    if (*stage) (void)hipHostFree(*stage);
    *stage = nullptr;
    *cap = 0;
    const size_t want = std::max(need, need + need / 4);
    if (hipHostMalloc((void**)stage, want, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      *stage = nullptr;
      return set_err(c, HBAM_ENOMEM, "hbam_records_to_host: hipHostMalloc(%zu) failed", want);
    }
    *cap = want;
  }
  uint64_t* roff;
  uint32_t* bad;
  int rc;
  if ((rc = ensure(c, B_RH_RECOFF, n + 1, &roff))) return rc;
  bad = (uint32_t*)(roff + n);
  HIPCHK(c, hipMemsetAsync(bad, 0, 4, c->stream));
  k_rebase_off<<<(uint32_t)std::min<uint64_t>(grid_for(n, 256), 16384), 256, 0, c->stream>>>(dv->rec_off, dv->block_size,
                                                                                             n, lo, roff, bad);
  HIPCHK(c, hipGetLastError());
  uint8_t* p = *stage;
  h->voffset = (uint64_t*)p;
  h->key = (int64_t*)(p + 8 * n);
  h->rec_off = (uint64_t*)(p + 16 * n);
  h->block_size = (int32_t*)(p + 24 * n);
  h->ubuf = p + cols;
  h->ubuf_len = hi - lo;
  HIPCHK(c, hipMemcpyAsync(h->voffset, dv->voffset, 8 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(h->key, dv->key, 8 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(h->rec_off, roff, 8 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(h->block_size, dv->block_size, 4 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(h->ubuf, dv->ubuf + lo, hi - lo, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->pinned_small + 3, bad, 4, hipMemcpyDeviceToHost, c->stream));
  const hipError_t e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    memset(h, 0, sizeof *h);
    return set_err(c, HBAM_EDEVICE, "hbam_records_to_host: %s", hipGetErrorString(e));
  }
  if ((uint32_t)c->pinned_small[3]) {
    memset(h, 0, sizeof *h);
    return set_err(c, HBAM_EINVAL, "hbam_records_to_host: records are not contiguous in ubuf (not a decoded split's "
                                   "columns)");
  }
  return HBAM_OK;
}
}  // namespace

// Records-only host copy for the drop-in reader (BAMRecordReader.nextKeyValue, :172-188, needs a
// record's bytes, its key and its file pointer): 28 B of columns per record + the records' bytes,
// into the context's pinned staging (one D2H pass at the DMA rate, no malloc per window).
extern "C" int hbam_records_to_host(hbam_ctx* c, const hbam_columns* dv, hbam_columns* h) {
  if (!c || !dv || !h) return HBAM_EINVAL;
  return records_to_host(c, dv, h, &c->rec_host, &c->rec_host_cap);
}

// The same into the split stream's own staging: each reader of a context keeps its window's host
// copy while other streams of the context read theirs
extern "C" int hbam_split_records_to_host(hbam_split_stream* s, const hbam_columns* dv, hbam_columns* h) {
  if (!s || !dv || !h) return HBAM_EINVAL;
  return records_to_host(s->c, dv, h, &s->rec_host, &s->rec_host_cap);
}

extern "C" void hbam_release_columns(hbam_ctx* c, hbam_columns* dv) {
  (void)c;
  if (dv) memset(dv, 0, sizeof *dv);
}

// =====================================================================================
// Guessers (kernels in hbam_guess.hip)
// =====================================================================================
namespace {
struct GuessWork {
  uint8_t* scratch;
  uint8_t* lens;
  uint8_t* bufs;
  int64_t *beg, *end, *out, *wlen;
  uint64_t* wptr;
  int32_t* err;
};
int guess_work(hbam_ctx* c, uint64_t k, GuessWork* w) {
  int rc;
  uint8_t* base;
  const uint64_t per = 65536 + LENS_SLOT + 8 + 8 * 5 + 4;
  if ((rc = ensure(c, B_G_WORK, k * per + 4096, &base))) return rc;
  w->scratch = base;
  w->lens = base + k * 65536;
  w->bufs = w->lens + k * LENS_SLOT;
  uint8_t* q = w->bufs + k * 8;
  q = (uint8_t*)(((uintptr_t)q + 15) & ~(uintptr_t)15);
  w->beg = (int64_t*)q;
  w->end = w->beg + k;
  w->out = w->end + k;
  w->wlen = w->out + k;
  w->wptr = (uint64_t*)(w->wlen + k);
  w->err = (int32_t*)(w->wptr + k);
  return HBAM_OK;
}

// Window block cache of a batch of guesses (see hbam_guess.hip): candidates, block records,
// batched inflate + CRC.  Fills the GCache arrays the guess kernel reads.
struct GuessCache {
  uint32_t* cn = nullptr;
  uint64_t *cbase = nullptr, *cpos = nullptr, *cuoff = nullptr;
  BlockRec* cblk = nullptr;
  uint8_t* cubuf = nullptr;
  int32_t* cst = nullptr;
  uint32_t* ccrc = nullptr;
};
int build_guess_cache(hbam_ctx* c, const GuessWork& w, uint64_t k, GuessCache* gc) {
  int rc;
  uint64_t* slots;
  uint32_t* cisz;
  if ((rc = ensure(c, B_G_CN, k + 1, &gc->cn))) return rc;
  if ((rc = ensure(c, B_G_CBASE, k + 1, &gc->cbase))) return rc;
  if ((rc = ensure(c, B_G_SLOTS, k * GC_CAP, &slots))) return rc;
  k_guess_cands<<<(uint32_t)k, 256, 0, c->stream>>>(w.wptr, w.wlen, w.beg, w.end, gc->cn, slots);
  HIPCHK(c, hipGetLastError());
  // windows over the cap contribute no cached blocks: clamp the counts for the scan
  uint32_t* cn_eff;
  if ((rc = ensure(c, B_G_CNEFF, k + 1, &cn_eff))) return rc;
  k_guess_clamp<<<grid_for(k, 256), 256, 0, c->stream>>>(gc->cn, (uint32_t)k, cn_eff);
  uint64_t ncand = 0;
  if ((rc = scan_exclusive<uint32_t>(c, cn_eff, k, gc->cbase, &ncand))) return rc;
  if ((rc = ensure(c, B_G_CPOS, ncand + 1, &gc->cpos))) return rc;
  if ((rc = ensure(c, B_G_CBLK, ncand + 1, &gc->cblk))) return rc;
  if ((rc = ensure(c, B_G_CISZ, ncand + 1, &cisz))) return rc;
  k_guess_cand_blocks<<<(uint32_t)k, 64, 0, c->stream>>>(w.wptr, w.wlen, w.beg, w.end, (uint32_t)k, gc->cn,
                                                        gc->cbase, slots, gc->cpos, gc->cblk, cisz);
  HIPCHK(c, hipGetLastError());
  uint64_t utotal = 0;
  if ((rc = ensure(c, B_G_CUOFF, ncand + 1, &gc->cuoff))) return rc;
  if ((rc = scan_exclusive<uint32_t>(c, cisz, ncand, gc->cuoff, &utotal))) return rc;
  if ((rc = ensure(c, B_G_CUBUF, utotal + UBUF_SLACK, &gc->cubuf))) return rc;
  if ((rc = ensure(c, B_G_CST, ncand + 1, &gc->cst))) return rc;
  if ((rc = ensure(c, B_G_CCRC, ncand + 1, &gc->ccrc))) return rc;
  // block records carry device addresses (windows live in different buffers): comp = null
  if (ncand)
    if ((rc = inflate_blocks(c, nullptr, gc->cblk, ncand, gc->cuoff, gc->cubuf, gc->cst, true, gc->ccrc)))
      return rc;
  return HBAM_OK;
}

// The window a guesser reads (BAMSplitGuesser.java:114-125 / BGZFSplitGuesser.java:62-63):
// min((int)(end - beg), cap) bytes from beg, cut at the end of the file.
uint64_t window_len(uint64_t file_len, int64_t beg, int64_t end, int64_t cap) {
  int32_t want = (int32_t)(end - beg);
  if (want > cap) want = (int32_t)cap;
  if (want <= 0 || beg < 0 || (uint64_t)beg > file_len) return 0;
  const uint64_t avail = file_len - (uint64_t)beg;
  return avail < (uint64_t)want ? avail : (uint64_t)want;
}

// k BAM guesses over device windows (wptr[i]: device address of file byte beg[i], wlen[i]
// bytes there), in launches of c->guess_batch.
int guess_run(hbam_ctx* c, const uint64_t* wptr, const int64_t* wlen, const int64_t* beg,
              const int64_t* end, uint64_t k, int32_t n_ref, int64_t* out, int32_t* err) {
  // Initial ByteBuffer of BAMSplitGuesser(ss, conf): the ctor reads the file magic into it
  // (:85-87) and throws unless it is 1f 8b 08 04.  Only windows shorter than 4 bytes could
  // observe a stale buffer carried over from a previous guess, and those always return `end`
  // (the XLEN seek at p0+10 fails), so guesses are independent.
  const uint8_t magic[8] = {0x1f, 0x8b, 0x08, 0x04, 0, 0, 0, 0};
  HIPCHK(c, hipEventRecord(c->ev[9], c->stream));
  uint64_t batch = c->guess_batch;
  int rc;
  for (uint64_t g0 = 0; g0 < k;) {
    const uint64_t kb = std::min(batch, k - g0);
    GuessWork w;
    if ((rc = guess_work(c, kb, &w))) {
      if (rc == HBAM_ENOMEM && kb > 1) {  // back off: half the guesses per launch
        batch = (kb + 1) / 2;
        continue;
      }
      return rc;
    }
    std::vector<uint8_t> ib(kb * 8);
    for (uint64_t i = 0; i < kb; ++i) memcpy(&ib[i * 8], magic, 8);
    HIPCHK(c, hipMemcpyAsync(w.bufs, ib.data(), kb * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(w.beg, beg + g0, kb * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(w.end, end + g0, kb * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(w.wptr, wptr + g0, kb * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(w.wlen, wlen + g0, kb * 8, hipMemcpyHostToDevice, c->stream));
    GuessCache gc;
    if ((rc = build_guess_cache(c, w, kb, &gc))) {
      if (rc == HBAM_ENOMEM && kb > 1) {
        batch = (kb + 1) / 2;
        continue;
      }
      return rc;
    }
    k_guess_bam_wave<<<(uint32_t)kb, 64, 0, c->stream>>>(
        w.wptr, w.wlen, w.beg, w.end, (uint32_t)kb, n_ref, w.scratch, w.lens, w.bufs, w.out,
        w.err, gc.cn, gc.cbase, gc.cpos, gc.cblk, gc.cuoff, gc.cubuf, gc.cst, gc.ccrc);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(out + g0, w.out, kb * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(err + g0, w.err, kb * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    g0 += kb;
  }
  HIPCHK(c, hipEventRecord(c->ev[10], c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->timing = hbam_timing{};
  c->timing.total_ms = ev_ms(c, 9, 10);
  return HBAM_OK;
}

// Windows of a whole file: views into a device-resident file, or (host file) the windows
// gathered on the host and staged alone — no guess call stages the file.
int file_windows(hbam_ctx* c, const uint8_t* file, int on_device, uint64_t file_len, const int64_t* beg,
                 const int64_t* end, uint64_t k, int64_t cap, std::vector<uint64_t>* wptr,
                 std::vector<int64_t>* wlen) {
  wptr->resize(k);
  wlen->resize(k);
  std::vector<uint64_t> woff(k + 1, 0);
  for (uint64_t i = 0; i < k; ++i) {
    (*wlen)[i] = (int64_t)window_len(file_len, beg[i], end[i], cap);
    woff[i + 1] = woff[i] + (uint64_t)(*wlen)[i];
  }
  if (on_device) {
    for (uint64_t i = 0; i < k; ++i)
      (*wptr)[i] = (uint64_t)(uintptr_t)(file + ((*wlen)[i] ? beg[i] : 0));
    return HBAM_OK;
  }
  uint8_t* dw;
  int rc;
  if ((rc = ensure(c, B_G_WIN, woff[k] + 64, &dw))) return rc;
  for (uint64_t i = 0; i < k; ++i) {
    if ((*wlen)[i])
      HIPCHK(c, hipMemcpyAsync(dw + woff[i], file + beg[i], (size_t)(*wlen)[i], hipMemcpyHostToDevice, c->stream));
    (*wptr)[i] = (uint64_t)(uintptr_t)(dw + woff[i]);
  }
  return HBAM_OK;
}

// Caller-gathered windows: window i = windows[win_off[i], win_off[i+1]), which must be exactly
// the bytes the guesser reads (window_len); staged to the device when on the host.
int caller_windows(hbam_ctx* c, const uint8_t* windows, int on_device, const uint64_t* win_off,
                   uint64_t file_len, const int64_t* beg, const int64_t* end, uint64_t k, int64_t cap,
                   std::vector<uint64_t>* wptr, std::vector<int64_t>* wlen) {
  wptr->resize(k);
  wlen->resize(k);
  if (win_off[0] != 0) return set_err(c, HBAM_EINVAL, "win_off[0] must be 0");
  for (uint64_t i = 0; i < k; ++i) {
    const uint64_t want = window_len(file_len, beg[i], end[i], cap);
    if (win_off[i + 1] < win_off[i] || win_off[i + 1] - win_off[i] != want)
      return set_err(c, HBAM_EINVAL, "window %llu holds %llu bytes, the guesser reads %llu",
                     (unsigned long long)i, (unsigned long long)(win_off[i + 1] - win_off[i]),
                     (unsigned long long)want);
    (*wlen)[i] = (int64_t)want;
  }
  const uint8_t* dw = windows;
  if (!on_device) {
    uint8_t* d;
    int rc;
    if ((rc = ensure(c, B_G_WIN, win_off[k] + 64, &d))) return rc;
    if (win_off[k]) HIPCHK(c, hipMemcpyAsync(d, windows, win_off[k], hipMemcpyHostToDevice, c->stream));
    dw = d;
  }
  for (uint64_t i = 0; i < k; ++i) (*wptr)[i] = (uint64_t)(uintptr_t)(dw + win_off[i]);
  return HBAM_OK;
}

}  // namespace

extern "C" uint64_t hbam_guess_window_len(uint64_t file_len, int64_t beg, int64_t end) {
  return window_len(file_len, beg, end, G_MAX_BYTES_READ);
}

extern "C" uint64_t hbam_guess_bgzf_window_len(uint64_t file_len, int64_t beg, int64_t end) {
  return window_len(file_len, beg, end, G_BGZF_WINDOW);
}

extern "C" int hbam_guess_batch(hbam_ctx* c, const uint8_t* file, int on_device, uint64_t file_len,
                                const int64_t* beg, const int64_t* end, uint64_t k, int32_t n_ref,
                                int64_t* out, int32_t* err) {
  if (!c || !file || (k && (!beg || !end || !out || !err))) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  if (k == 0) return HBAM_OK;
  std::vector<uint64_t> wp;
  std::vector<int64_t> wl;
  int rc = file_windows(c, file, on_device, file_len, beg, end, k, G_MAX_BYTES_READ, &wp, &wl);
  if (rc) return rc;
  return guess_run(c, wp.data(), wl.data(), beg, end, k, n_ref, out, err);
}

extern "C" int hbam_guess_windows(hbam_ctx* c, const uint8_t* windows, int on_device,
                                  const uint64_t* win_off, uint64_t file_len, const int64_t* beg,
                                  const int64_t* end, uint64_t k, int32_t n_ref, int64_t* out,
                                  int32_t* err) {
  if (!c || (k && (!windows || !win_off || !beg || !end || !out || !err))) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  if (k == 0) return HBAM_OK;
  std::vector<uint64_t> wp;
  std::vector<int64_t> wl;
  int rc = caller_windows(c, windows, on_device, win_off, file_len, beg, end, k, G_MAX_BYTES_READ, &wp, &wl);
  if (rc) return rc;
  return guess_run(c, wp.data(), wl.data(), beg, end, k, n_ref, out, err);
}

extern "C" int64_t hbam_guess_bam_record_start(hbam_ctx* c, const uint8_t* file, int on_device,
                                               uint64_t file_len, int64_t beg, int64_t end,
                                               int32_t n_ref, int32_t* err) {
  int64_t out = end;
  int32_t e = HBAM_OK;
  const int rc = hbam_guess_batch(c, file, on_device, file_len, &beg, &end, 1, n_ref, &out, &e);
  if (err) *err = rc ? rc : e;
  return out;
}

namespace {
int64_t guess_bgzf_run(hbam_ctx* c, uint64_t wptr, int64_t wlen, int64_t beg, int64_t end, int32_t* err) {
  GuessWork w;
  int rc = guess_work(c, 1, &w);
  if (rc) {
    if (err) *err = rc;
    return end;
  }
  int64_t out = end;
  int32_t e = HBAM_OK;
  if (hipMemcpyAsync(w.beg, &beg, 8, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(w.end, &end, 8, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(w.wptr, &wptr, 8, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(w.wlen, &wlen, 8, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
    if (err) *err = HBAM_EDEVICE;
    return end;
  }
  k_guess_bgzf<<<1, GUESS_WG, 0, c->stream>>>(w.wptr, w.wlen, w.beg, w.end, 1, w.scratch, w.lens, w.out, w.err);
  if (hipMemcpyAsync(&out, w.out, 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipMemcpyAsync(&e, w.err, 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess) {
    if (err) *err = HBAM_EDEVICE;
    return end;
  }
  if (err) *err = e;
  return out;
}
}  // namespace

extern "C" int64_t hbam_guess_bgzf_block_start(hbam_ctx* c, const uint8_t* file, int on_device,
                                               uint64_t file_len, int64_t beg, int64_t end,
                                               int32_t* err) {
  if (!c || !file) {
    if (err) *err = HBAM_EINVAL;
    return end;
  }
  if (hipSetDevice(c->device) != hipSuccess) {
    if (err) *err = HBAM_EDEVICE;
    return end;
  }
  std::vector<uint64_t> wp;
  std::vector<int64_t> wl;
  const int rc = file_windows(c, file, on_device, file_len, &beg, &end, 1, G_BGZF_WINDOW, &wp, &wl);
  if (rc) {
    if (err) *err = rc;
    return end;
  }
  return guess_bgzf_run(c, wp[0], wl[0], beg, end, err);
}

extern "C" int64_t hbam_guess_bgzf_window(hbam_ctx* c, const uint8_t* window, int on_device, uint64_t wlen,
                                          uint64_t file_len, int64_t beg, int64_t end, int32_t* err) {
  if (!c || (!window && wlen)) {
    if (err) *err = HBAM_EINVAL;
    return end;
  }
  if (hipSetDevice(c->device) != hipSuccess) {
    if (err) *err = HBAM_EDEVICE;
    return end;
  }
  const uint64_t off[2] = {0, wlen};
  std::vector<uint64_t> wp;
  std::vector<int64_t> wl;
  const uint8_t* w = window ? window : (const uint8_t*)off;  // any address for an empty window
  const int rc = caller_windows(c, w, on_device, off, file_len, &beg, &end, 1, G_BGZF_WINDOW, &wp, &wl);
  if (rc) {
    if (err) *err = rc;
    return end;
  }
  return guess_bgzf_run(c, wp[0], wl[0], beg, end, err);
}

// BAMInputFormat.addProbabilisticSplits (BAMInputFormat.java:163-224) for one file, from the
// guesses of its FileSplits (the loop after the guesser calls).
namespace {
int64_t splits_from_guesses(hbam_ctx* c, const uint64_t* end, uint64_t n, const int64_t* g,
                            const int32_t* er, uint64_t* v_start, uint64_t* v_end) {
  int64_t out = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (er[i]) return set_err(c, er[i], "guesser raised an exception for split %llu", (unsigned long long)i);
    const uint64_t aligned_end = end[i] << 16 | 0xffff;
    if (g[i] == (int64_t)end[i]) {
      if (out == 0) return set_err(c, HBAM_EIO, "no reads in first split: bad BAM file or tiny split size?");
      v_end[out - 1] = aligned_end;
    } else {
      v_start[out] = (uint64_t)g[i];
      v_end[out] = aligned_end;
      ++out;
    }
  }
  return out;
}
// BAMSplitGuesser(ss, conf) ctor over the file's first head_len bytes: the header (n_ref) and
// the magic check.  A prefix too short for the header -> HBAM_ETRUNC (read more and retry).
int guesser_ctor(hbam_ctx* c, const uint8_t* head, int on_device, uint64_t head_len, uint64_t file_len,
                 int32_t* n_ref) {
  hbam_header h;
  int rc = hbam_parse_header(c, head, on_device, head_len, &h);
  if (rc) return (rc == HBAM_EFORMAT && head_len < file_len) ? set_err(c, HBAM_ETRUNC, "header prefix too short") : rc;
  uint8_t m[4] = {0, 0, 0, 0};
  if (head_len >= 4) {
    if (on_device) {
      HIPCHK(c, hipMemcpyAsync(c->pinned_small, head, 4, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      memcpy(m, c->pinned_small, 4);
    } else {
      memcpy(m, head, 4);
    }
  }
  if (head_len < 4 || !(m[0] == 0x1f && m[1] == 0x8b && m[2] == 8 && m[3] == 4))
    return set_err(c, HBAM_EFORMAT, "Does not seem like a BAM file");
  *n_ref = h.n_ref;
  return HBAM_OK;
}
}  // namespace

extern "C" int64_t hbam_probabilistic_splits(hbam_ctx* c, const uint8_t* file, int on_device,
                                             uint64_t file_len, const uint64_t* beg,
                                             const uint64_t* end, uint64_t n, uint64_t* v_start,
                                             uint64_t* v_end) {
  if (!c || !file || (n && (!beg || !end || !v_start || !v_end))) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  // the header from a growing prefix (the file itself is never staged whole)
  int32_t n_ref = 0;
  int rc;
  for (uint64_t hl = std::min<uint64_t>(file_len, 1 << 20);; hl = std::min<uint64_t>(file_len, 4 * hl)) {
    rc = guesser_ctor(c, file, on_device, hl, file_len, &n_ref);
    if (rc != HBAM_ETRUNC || hl == file_len) break;
  }
  if (rc) return rc;
  std::vector<int64_t> b(n), e(n), g(n);
  std::vector<int32_t> er(n);
  for (uint64_t i = 0; i < n; ++i) {
    b[i] = (int64_t)beg[i];
    e[i] = (int64_t)end[i];
  }
  if ((rc = hbam_guess_batch(c, file, on_device, file_len, b.data(), e.data(), n, n_ref, g.data(), er.data())))
    return rc;
  return splits_from_guesses(c, end, n, g.data(), er.data(), v_start, v_end);
}

extern "C" int64_t hbam_probabilistic_splits_windows(hbam_ctx* c, const uint8_t* head, uint64_t head_len,
                                                     const uint8_t* windows, int on_device,
                                                     const uint64_t* win_off, uint64_t file_len,
                                                     const uint64_t* beg, const uint64_t* end, uint64_t n,
                                                     uint64_t* v_start, uint64_t* v_end) {
  if (!c || !head || (n && (!windows || !win_off || !beg || !end || !v_start || !v_end))) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  int32_t n_ref = 0;
  int rc = guesser_ctor(c, head, 0, head_len, file_len, &n_ref);
  if (rc) return rc;
  std::vector<int64_t> b(n), e(n), g(n);
  std::vector<int32_t> er(n);
  for (uint64_t i = 0; i < n; ++i) {
    b[i] = (int64_t)beg[i];
    e[i] = (int64_t)end[i];
  }
  if ((rc = hbam_guess_windows(c, windows, on_device, win_off, file_len, b.data(), e.data(), n, n_ref, g.data(),
                               er.data())))
    return rc;
  return splits_from_guesses(c, end, n, g.data(), er.data(), v_start, v_end);
}

// ---- Sort plugin path (Sort.java:84-188) -----------------------------
extern "C" int hbam_sort_keys(hbam_ctx* c, const int64_t* keys, uint64_t n, int64_t* keys_out,
                              uint32_t* perm) {
  if (!c || (n && (!keys || !perm))) return HBAM_EINVAL;
  if (n > 0xffffffffull) return set_err(c, HBAM_EINVAL, "hbam_sort_keys: n > 2^32-1");
  HIPCHK(c, hipSetDevice(c->device));
  c->timing = hbam_timing{};
  if (n == 0) return HBAM_OK;
  const uint32_t ntiles = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
  uint64_t *k0, *k1, *off;
  uint32_t *v0, *v1, *cnt, *hist;
  int rc;
  if ((rc = ensure(c, B_S_UK0, n, &k0)) || (rc = ensure(c, B_S_UK1, n, &k1)) ||
      (rc = ensure(c, B_S_V0, n, &v0)) || (rc = ensure(c, B_S_V1, n, &v1)) ||
      (rc = ensure(c, B_S_CNT, (uint64_t)ntiles * 256, &cnt)) ||
      (rc = ensure(c, B_S_OFF, (uint64_t)ntiles * 256 + 1, &off)) ||
      (rc = ensure(c, B_S_HIST, 8 * 256, &hist)))
    return rc;
  HIPCHK(c, hipEventRecord(c->ev[9], c->stream));
  HIPCHK(c, hipMemsetAsync(hist, 0, 8 * 256 * 4, c->stream));
  const uint32_t ig = (uint32_t)std::min<uint64_t>(grid_for(n, RS_WG), 2048);
  k_rs_init<<<ig, RS_WG, 0, c->stream>>>(keys, n, k0, v0, hist);
  HIPCHK(c, hipGetLastError());
  std::vector<uint32_t> h(8 * 256);
  HIPCHK(c, copy_sync(c, h.data(), hist, h.size() * 4, hipMemcpyDeviceToHost));
  uint64_t* kin = k0;
  uint64_t* kout = k1;
  uint32_t* vin = v0;
  uint32_t* vout = v1;
  int passes = 0;
  for (uint32_t d = 0; d < 8; ++d) {
    bool trivial = false;
    for (uint32_t b = 0; b < 256; ++b) trivial |= (h[d * 256 + b] == n);
    if (trivial) continue;  // every key has the same digit: the pass is the identity
    const uint32_t shift = 8 * d;
    k_rs_count<<<ntiles, RS_WG, 0, c->stream>>>(kin, n, shift, ntiles, cnt);
    HIPCHK(c, hipGetLastError());
    if ((rc = scan_exclusive(c, cnt, (uint64_t)ntiles * 256, off, nullptr))) return rc;
    k_rs_scatter<<<ntiles, RS_WG, 0, c->stream>>>(kin, vin, n, shift, ntiles, off, kout, vout);
    HIPCHK(c, hipGetLastError());
    std::swap(kin, kout);
    std::swap(vin, vout);
    ++passes;
  }
  HIPCHK(c, hipMemcpyAsync(perm, vin, n * 4, hipMemcpyDeviceToDevice, c->stream));
  if (keys_out) k_rs_finish<<<grid_for(n, RS_WG), RS_WG, 0, c->stream>>>(kin, n, keys_out);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->ev[10], c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->timing.total_ms = ev_ms(c, 9, 10);
  c->timing.n_records = n;
  c->timing.n_blocks = (uint64_t)passes;  // radix passes actually run
  return HBAM_OK;
}

extern "C" int hbam_gather_records(hbam_ctx* c, const uint8_t* ubuf, const uint64_t* rec_off,
                                   const int32_t* block_size, const uint32_t* perm, uint64_t n,
                                   uint8_t* out, uint64_t out_cap, uint64_t* out_off,
                                   uint64_t* total_bytes) {
  if (!c || !out_off || (n && !block_size) || (out && n && (!ubuf || !rec_off))) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  uint32_t* lens;
  if ((rc = ensure(c, B_S_LENS, n + 1, &lens))) return rc;
  HIPCHK(c, hipEventRecord(c->ev[9], c->stream));
  if (n) k_perm_lens<<<grid_for(n, RS_WG), RS_WG, 0, c->stream>>>(block_size, perm, n, lens);
  HIPCHK(c, hipGetLastError());
  uint64_t tot = 0;
  if ((rc = scan_exclusive(c, lens, n, out_off, &tot))) return rc;
  if (total_bytes) *total_bytes = tot;
  if (!out) return HBAM_OK;  // size query
  if (tot > out_cap) return set_err(c, HBAM_EINVAL, "hbam_gather_records: %llu bytes > out_cap %llu",
                                    (unsigned long long)tot, (unsigned long long)out_cap);
  if (n) {
    // one wave per record, grid-stride: a grid of 64 x n threads would pass 2^32 above 67 M
    // records (the dispatch packet's grid size is 32-bit)
    // a wave per 64-record tile (A/B against the wave-per-record gather: profiles/r04/ab/)
    k_gather_records_tile<<<(uint32_t)std::min<uint64_t>((n + 255) / 256, POOLS_MAX_WG), 256, 0, c->stream>>>(
        ubuf, rec_off, perm, n, out_off, out);
  }
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->ev[10], c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->timing.pools_ms = ev_ms(c, 9, 10);
  c->timing.pool_bytes = tot;
  return HBAM_OK;
}

extern "C" int hbam_permute(hbam_ctx* c, const void* src, uint32_t elem_size, const uint32_t* perm,
                            uint64_t n, void* out) {
  if (!c || (n && (!src || !perm || !out)) || (elem_size != 4 && elem_size != 8)) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  if (n) {
    if (elem_size == 8)
      k_permute<uint64_t><<<grid_for(n, RS_WG), RS_WG, 0, c->stream>>>((const uint64_t*)src, perm, n,
                                                                        (uint64_t*)out);
    else
      k_permute<uint32_t><<<grid_for(n, RS_WG), RS_WG, 0, c->stream>>>((const uint32_t*)src, perm, n,
                                                                        (uint32_t*)out);
  }
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return HBAM_OK;
}

extern "C" int hbam_device_alloc(hbam_ctx* c, uint64_t bytes, void** dev_out) {
  if (!c || !dev_out) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  void* d = nullptr;
  // + 64 readable bytes past the end: a buffer from here may be handed back as a device input,
  // which the kernels read in whole 16-byte quads and 28-32-byte windows (include/hbam.h)
  if (hipMalloc(&d, bytes + 64) != hipSuccess) {
    (void)hipGetLastError();
    return set_err(c, HBAM_ENOMEM, "hbam_device_alloc(%llu) failed", (unsigned long long)bytes);
  }
  *dev_out = d;
  return HBAM_OK;
}

namespace {
// sorted run of n records whose bytes sit at ubuf[rec_off[i]] (block_size[i] + 4 bytes each)
int sort_run(hbam_ctx* c, const int64_t* key, const uint64_t* voffset, const int32_t* block_size,
             const uint8_t* ubuf, const uint64_t* rec_off, uint64_t n, hbam_sorted_run* out) {
  int rc;
  uint64_t total = 0;
  if (!out->payload) {  // size query
    uint64_t* off;
    if ((rc = ensure(c, B_S_OFF, n + 1, &off))) return rc;
    if ((rc = hbam_gather_records(c, ubuf, rec_off, block_size, nullptr, n, nullptr, 0, off, &total)))
      return rc;
    out->n = n;
    out->payload_bytes = total;
    return HBAM_OK;
  }
  if (n && (!out->key || !out->voffset || !out->block_size || !out->offsets)) return HBAM_EINVAL;
  uint32_t* perm;
  if ((rc = ensure(c, B_S_PERM, n + 1, &perm))) return rc;
  if ((rc = hbam_sort_keys(c, key, n, out->key, perm))) return rc;
  if ((rc = hbam_permute(c, voffset, 8, perm, n, out->voffset))) return rc;
  if ((rc = hbam_permute(c, block_size, 4, perm, n, out->block_size))) return rc;
  if ((rc = hbam_gather_records(c, ubuf, rec_off, block_size, perm, n, out->payload,
                                out->payload_bytes, out->offsets, &total)))
    return rc;
  out->n = n;
  out->payload_bytes = total;
  return HBAM_OK;
}
}  // namespace

extern "C" int hbam_sort_split(hbam_ctx* c, const hbam_columns* dv, hbam_sorted_run* out) {
  if (!c || !dv || !out) return HBAM_EINVAL;
  if (dv->status != HBAM_OK) return set_err(c, dv->status, "hbam_sort_split: the decode raised %d", dv->status);
  HIPCHK(c, hipSetDevice(c->device));
  return sort_run(c, dv->key, dv->voffset, dv->block_size, dv->ubuf, dv->rec_off, dv->n_records, out);
}

extern "C" int hbam_merge_remap(hbam_ctx* c, hbam_columns* dv, const int32_t* ref_map, int32_t n_in,
                                uint64_t* bad_record) {
  if (!c || !dv || !bad_record || n_in < 0 || (n_in && !ref_map)) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  *bad_record = ~0ull;
  const uint64_t n = dv->n_records;
  if (n == 0) return HBAM_OK;
  int32_t* dmap;
  uint64_t* err;
  int rc;
  if ((rc = ensure(c, B_M_ERR, 1, &err))) return rc;
  if ((rc = ensure(c, B_M_MAP, (uint64_t)n_in + 1, &dmap))) return rc;
  HIPCHK(c, hipMemsetAsync(err, 0xff, 8, c->stream));
  if (n_in) HIPCHK(c, hipMemcpyAsync(dmap, ref_map, 4ull * n_in, hipMemcpyHostToDevice, c->stream));
  k_merge_remap<<<grid_for(n, RS_WG), RS_WG, 0, c->stream>>>(dv->ubuf, dv->rec_off, n, dv->ref_id, dv->next_ref_id,
                                                            dv->key, dv->flag, dv->pos, dmap, n_in,
                                                            (unsigned long long*)err);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, copy_sync(c, bad_record, err, 8, hipMemcpyDeviceToHost));
  return HBAM_OK;
}

extern "C" int hbam_sort_received(hbam_ctx* c, const int64_t* key, const int64_t* voffset,
                                  const int32_t* block_size, const uint8_t* payload, uint64_t n,
                                  hbam_sorted_run* out) {
  if (!c || !out || (n && (!key || !voffset || !block_size || !payload))) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  // record offsets of the received payload: exclusive scan of 4 + block_size
  uint64_t* rec_off;
  int rc;
  if ((rc = ensure(c, B_S_RECOFF, n + 1, &rec_off))) return rc;
  uint64_t total = 0;
  if ((rc = hbam_gather_records(c, nullptr, nullptr, block_size, nullptr, n, nullptr, 0, rec_off, &total)))
    return rc;
  return sort_run(c, key, (const uint64_t*)voffset, block_size, payload, rec_off, n, out);
}

extern "C" int hbam_sort_partition(hbam_ctx* c, const hbam_sorted_run* run, const int64_t* split_points,
                                   uint32_t nparts, uint64_t* rec_bounds, uint64_t* byte_bounds) {
  if (!c || !run || !rec_bounds || !byte_bounds || nparts == 0 || (nparts > 1 && !split_points))
    return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  const uint32_t m = nparts - 1;
  rec_bounds[0] = 0;
  byte_bounds[0] = 0;
  rec_bounds[nparts] = run->n;
  byte_bounds[nparts] = run->payload_bytes;
  if (m == 0) return HBAM_OK;
  if (run->n && (!run->key || !run->offsets)) return HBAM_EINVAL;
  uint64_t* d;
  int rc;
  if ((rc = ensure(c, B_S_BOUNDS, 3 * (uint64_t)m, &d))) return rc;
  int64_t* dsp = (int64_t*)(d + 2 * (uint64_t)m);
  HIPCHK(c, hipMemcpyAsync(dsp, split_points, 8ull * m, hipMemcpyHostToDevice, c->stream));
  if (run->n) {
    k_sort_bounds<<<grid_for(m, RS_WG), RS_WG, 0, c->stream>>>(run->key, run->n, dsp, m, run->offsets, d,
                                                               d + m);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(rec_bounds + 1, d, 8ull * m, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(byte_bounds + 1, d + m, 8ull * m, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  } else {
    for (uint32_t j = 1; j < nparts; ++j) rec_bounds[j] = byte_bounds[j] = 0;
  }
  return HBAM_OK;
}

extern "C" int64_t hbam_splitting_index(hbam_ctx* c, const hbam_columns* dv, int32_t granularity,
                                       uint64_t file_len, uint64_t* out, uint64_t cap) {
  if (!c || !dv || !out || granularity <= 0) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  const uint64_t n = dv->n_records;
  if (n == 0 && dv->status == HBAM_OK)
    return set_err(c, HBAM_EINVAL, "hbam_splitting_index: the split holds no record (first voffset unknown)");
  if (dv->status != HBAM_OK) return set_err(c, dv->status, "hbam_splitting_index: decode raised %d", dv->status);
  const uint64_t k = n / (uint64_t)granularity;
  const uint64_t total = k + 2;
  if (total > cap) return set_err(c, HBAM_EINVAL, "hbam_splitting_index: %llu entries > cap %llu",
                                  (unsigned long long)total, (unsigned long long)cap);
  uint64_t* d;
  int rc;
  if ((rc = ensure(c, B_S_OFF, k + 1, &d))) return rc;
  if (k) k_index_pick<<<grid_for(k, RS_WG), RS_WG, 0, c->stream>>>(dv->voffset, n, (uint32_t)granularity, d);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, copy_sync(c, out, dv->voffset, 8, hipMemcpyDeviceToHost));
  HIPCHK(c, copy_sync(c, out + 1, d, 8 * k, hipMemcpyDeviceToHost));
  out[k + 1] = file_len << 16;
  return (int64_t)total;
}

extern "C" int64_t hbam_bgzf_block_index(hbam_ctx* c, const uint8_t* file, int on_device,
                                        uint64_t len, int32_t granularity, uint64_t* out,
                                        uint64_t cap) {
  if (!c || (!file && len) || !out || granularity <= 0) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  if (len == 0) {  // no block: only the terminating file length (:124-125)
    if (cap < 1) return set_err(c, HBAM_EINVAL, "hbam_bgzf_block_index: cap 0");
    out[0] = 0;
    return 1;
  }
  const uint8_t* d;
  int rc = stage_comp(c, file, on_device, len, &d);
  if (rc) return rc;
  Chain ch;
  if ((rc = build_chain(c, d, len, 0, true, &ch))) return rc;
  if (ch.end_code != HBAM_EEOF)  // skipBlock's ioError (:133-180)
    return set_err(c, HBAM_EIO, "hbam_bgzf_block_index: no BGZF block at %llu",
                   (unsigned long long)ch.end_pos);
  const uint64_t k = ch.nb / (uint64_t)granularity;
  if (k + 1 > cap) return set_err(c, HBAM_EINVAL, "hbam_bgzf_block_index: %llu entries > cap %llu",
                                  (unsigned long long)(k + 1), (unsigned long long)cap);
  if (k) {
    uint64_t* dout;
    if ((rc = ensure(c, B_S_OFF, k, &dout))) return rc;
    k_bgzfi_pick<<<grid_for(k, RS_WG), RS_WG, 0, c->stream>>>((const BlockRec*)c->bufs[B_BLK].p, ch.nb,
                                                              len, (uint32_t)granularity, k, dout);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, copy_sync(c, out, dout, 8 * k, hipMemcpyDeviceToHost));
  }
  out[k] = len & 0xffffffffffffull;
  return (int64_t)(k + 1);
}

extern "C" int hbam_resolve_tokens(hbam_ctx* c, uint8_t* io, uint32_t isize, const uint32_t* bitmap,
                                   uint32_t tail_token, uint32_t tail_dist, int32_t* status) {
  if (!c || !io || !bitmap || !status || isize == 0 || isize > 65536u) return HBAM_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  BlockRec* blk;
  uint64_t* uoff;
  uint8_t* ub;
  uint32_t *bm, *tails;
  int32_t* st;
  int rc;
  if ((rc = ensure(c, B_BLK, 1, &blk)) || (rc = ensure(c, B_UOFF, 2, &uoff)) ||
      (rc = ensure(c, B_UBUF, isize + UBUF_SLACK, &ub)) || (rc = ensure(c, B_BITMAP, BITMAP_WORDS, &bm)) ||
      (rc = ensure(c, B_TAILS, 2, &tails)) || (rc = ensure(c, B_INFST, 1, &st)))
    return rc;
  BlockRec r{};
  r.isize = isize;
  r.clen = 26;
  const uint64_t uo[2] = {0, isize};
  const uint32_t tl[2] = {tail_token, tail_dist};
  const int32_t zero = INF_OK;
  HIPCHK(c, hipMemsetAsync(ub, 0, isize + UBUF_SLACK, c->stream));
  HIPCHK(c, hipMemsetAsync(bm, 0, BITMAP_WORDS * 4, c->stream));
  HIPCHK(c, hipMemcpyAsync(blk, &r, sizeof r, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(uoff, uo, sizeof uo, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(ub, io, isize, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(bm, bitmap, 4ull * ((isize + 31u) / 32u), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(tails, tl, sizeof tl, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(st, &zero, 4, hipMemcpyHostToDevice, c->stream));
  k_resolve_units<<<1, 64, 0, c->stream>>>(blk, uoff, 1, ub, bm, tails, st);
  HIPCHK(c, hipGetLastError());
  int32_t hs = 0;
  HIPCHK(c, hipMemcpyAsync(&hs, st, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(io, ub, isize, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  *status = hs == INF_OK ? HBAM_OK : HBAM_EDATA;
  return HBAM_OK;
}

#ifdef HBAM_PROF
// Profiling build only: attach a device buffer of 16 u64 per block for the per-block cycle
// counters of k_inflate_tokens / k_resolve (tools/profile_inflate.py --prof).
extern "C" int hbam_prof_attach(void* dev) {
  unsigned long long* p = (unsigned long long*)dev;
  return hipMemcpyToSymbol(HIP_SYMBOL(hbam::g_prof), &p, sizeof p) == hipSuccess ? 0 : -1;
}
extern "C" int hbam_prof_attach_deflate(void* dev) {
  unsigned long long* p = (unsigned long long*)dev;
  return hipMemcpyToSymbol(HIP_SYMBOL(hbam::g_dfprof), &p, sizeof p) == hipSuccess ? 0 : -1;
}
extern "C" int hbam_prof_attach_trace(void* dev, unsigned int idx) {
  unsigned long long* p = (unsigned long long*)dev;
  if (hipMemcpyToSymbol(HIP_SYMBOL(hbam::g_gtrace_idx), &idx, sizeof idx) != hipSuccess) return -1;
  return hipMemcpyToSymbol(HIP_SYMBOL(hbam::g_gtrace), &p, sizeof p) == hipSuccess ? 0 : -1;
}
extern "C" int hbam_prof_attach_guess(void* dev) {
  unsigned long long* p = (unsigned long long*)dev;
  return hipMemcpyToSymbol(HIP_SYMBOL(hbam::g_gprof), &p, sizeof p) == hipSuccess ? 0 : -1;
}
#endif

// =====================================================================================
// BGZF compression (hbam_deflate.hip): BlockCompressedOutputStream for the BAM writer.
namespace {
constexpr uint32_t DF_BATCH = 4096;  // blocks per launch: ~1 GiB of token scratch
}

extern "C" uint64_t hbam_bgzf_bound(uint64_t n, uint32_t block_size) {
  const uint32_t bs = block_size ? block_size : hbam::DF_MAXB;
  return ((n + bs - 1) / bs) * (uint64_t)hbam::DF_SLOT;
}

extern "C" int64_t hbam_bgzf_compress(hbam_ctx* c, const uint8_t* src, int src_on_device, uint64_t n,
                                      uint32_t block_size, uint8_t* dst, int dst_on_device, uint64_t dst_cap) {
  if (!c || (n && (!src || !dst))) return HBAM_EINVAL;
  const uint32_t bs = block_size ? block_size : DF_MAXB;
  if (bs > DF_MAXB || bs < 1024) return set_err(c, HBAM_EINVAL, "block_size %u not in [1024, %u]", bs, DF_MAXB);
  HIPCHK(c, hipSetDevice(c->device));
  if (n == 0) return 0;
  const uint8_t* d;
  int rc;
  if (src_on_device) {
    d = src;
  } else {
    uint8_t* ds;
    if ((rc = ensure(c, B_DF_SRC, n + 64, &ds))) return rc;
    HIPCHK(c, hipMemcpyAsync(ds, src, n, hipMemcpyHostToDevice, c->stream));
    d = ds;
  }
  const uint64_t nb = (n + bs - 1) / bs;
  uint64_t out_total = 0;
  HIPCHK(c, hipEventRecord(c->ev[9], c->stream));
  for (uint64_t b0 = 0; b0 < nb; b0 += DF_BATCH) {
    const uint32_t k = (uint32_t)std::min<uint64_t>(DF_BATCH, nb - b0);
    const uint64_t off0 = b0 * bs;
    const uint64_t nn = std::min<uint64_t>(n - off0, (uint64_t)k * bs);
    uint32_t *tok, *ntok, *crc, *csize;
    uint8_t* slots;
    uint64_t* off;
    if ((rc = ensure(c, B_DF_TOK, (uint64_t)k * bs, &tok)) || (rc = ensure(c, B_DF_NTOK, k, &ntok)) ||
        (rc = ensure(c, B_DF_CRC, k, &crc)) ||
        (rc = ensure(c, B_DF_SLOTS, (uint64_t)k * DF_SLOT, &slots)) || (rc = ensure(c, B_DF_CSIZE, k + 1, &csize)) ||
        (rc = ensure(c, B_DF_OFF, k + 1, &off)))
      return rc;
    k_crc_blocks<<<grid_for(k, 256), 256, 0, c->stream>>>(d + off0, nn, bs, k, crc);
    k_lz77_tokens<<<k, DF_WG, 0, c->stream>>>(d + off0, nn, bs, k, tok, ntok);
    k_deflate_encode<<<k, DF_WG, 0, c->stream>>>(d + off0, nn, bs, k, tok, ntok, crc, slots, csize);
    HIPCHK(c, hipGetLastError());
    uint64_t bytes = 0;
    if ((rc = scan_exclusive<uint32_t>(c, csize, k, off, &bytes))) return rc;
    if (out_total + bytes > dst_cap)
      return set_err(c, HBAM_EINVAL, "dst_cap %llu < %llu compressed bytes", (unsigned long long)dst_cap,
                     (unsigned long long)(out_total + bytes));
    uint8_t* pd;
    if (dst_on_device) {
      pd = dst + out_total;
    } else {
      if ((rc = ensure(c, B_DF_DST, bytes + 64, &pd))) return rc;
    }
    k_pack_members<<<k, 256, 0, c->stream>>>(slots, csize, off, k, pd);
    HIPCHK(c, hipGetLastError());
    if (!dst_on_device) HIPCHK(c, hipMemcpyAsync(dst + out_total, pd, bytes, hipMemcpyDeviceToHost, c->stream));
    out_total += bytes;
  }
  HIPCHK(c, hipEventRecord(c->ev[10], c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->timing = hbam_timing{};
  c->timing.total_ms = ev_ms(c, 9, 10);
  c->timing.ubuf_bytes = n;
  c->timing.comp_bytes = out_total;
  c->timing.n_blocks = nb;
  return (int64_t)out_total;
}

#include "hbam_consumers.hip"
#include "hbam_groups.hip"
#include "hbam_bcf_api.hip"
#include "hbam_comm.hip"
