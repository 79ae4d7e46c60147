// resolve_dev.h — LZ77 resolution (phase 2 of the batched inflate), one wave per BGZF block.
//
// Input (left in ubuf by k_inflate_tokens): literals at their final offsets, a 3-byte
// descriptor (len-3, dist-1 as u8 + u16 LE) at the first bytes of every match of >= 3 bytes,
// one bit per match start in the block's bitmap, and an optional final match of < 3 bytes
// (`tails`).  Output: the block's inflated bytes, in place.
//
// The block is walked in stretches of RS_S output bytes.  LDS holds a window of the RS_W
// bytes before the stretch, the stretch and the next stretch (matches spill up to 258 bytes
// past their stretch), ~12 KiB per wave in all (with the record list), so ~13 blocks share a CU.  Per stretch:
//   1. the stretch's match starts come from 64 bitmap words (one per lane), their
//      descriptors are read once into an LDS record list and split into
//        - "pre" matches: source ends before the stretch — every source byte is final —
//          copied all in parallel, reading the window in LDS or (source older than the
//          window, already written back) ubuf in global memory;
//        - "ordered" matches: source ends inside the stretch; executed in order in batches,
//          a batch = the longest prefix of the pending matches whose sources end before the
//          first pending destination (so every source byte is final), one lane per match;
//   2. the stretch is written back to ubuf and the window slides by RS_S.
// Raw stretch bytes and bitmap words are prefetched two / one stretch ahead.
#pragma once
#include <stdint.h>

namespace hbam {

#ifndef HBAM_RS_W
// A/B at 2 GB (stretch 2 KiB): 4096 -> 20.0 ms, 2048 -> 18.0, 1024 -> 16.7; at 10 GB with packed
// match records and 8 waves/SIMD (HBAM_RS_WAVES): 1024 -> 48.8 ms (LDS caps it at 7 waves), 512 ->
// 42.6 ms (profiles/r02/s2/ab_resolve_occupancy_10g.txt); 0 is not supported
#define HBAM_RS_W 512
#endif
#ifndef HBAM_RS_S
#define HBAM_RS_S 1024  // A/B at 2 GB (window 1 KiB): 2048 -> 16.8 ms, 1024 -> 11.7 ms
#endif
constexpr uint32_t RS_S = HBAM_RS_S;                  // stretch (output bytes): 1024 or 2048
constexpr uint32_t RS_C = RS_S / 1024;                // 16-byte columns per lane per stretch
constexpr uint32_t RS_W = HBAM_RS_W;                  // window kept in LDS behind the stretch
constexpr uint32_t RS_BUF = RS_W + 2 * RS_S + 48;     // + pad for 32-byte over-reads
static_assert(RS_W >= 16 && RS_W % 16 == 0 && (RS_S == 1024 || RS_S == 2048),
              "window: whole 16-byte columns; stretch: 1 or 2 KiB (one or two columns per lane)");
constexpr uint32_t RS_MAXM = RS_S / 3 + 2;            // matches starting in one stretch
constexpr uint32_t RS_PW = (RS_S + 16 + 258 + 31) / 32 + 1;  // pending-byte words of a stretch + spill

constexpr uint32_t RS_SLOTS = (RS_MAXM + 63) / 64;      // ordered matches per lane, at most
static_assert(RS_MAXM <= 512, "packed match records hold a 9-bit s_pos index");

// packed match record (s_pos index | len-3 << 9 | dist-1 << 17) -> p | len << 16 | dist << 32 |
// e << 48, e = the end of the match's external source (p - dist + min(len, dist))
__device__ __forceinline__ uint64_t rs_unpack(uint32_t pk, const uint16_t* s_pos) {
  const uint32_t p = s_pos[pk & 511u];
  const uint32_t len = ((pk >> 9) & 255u) + 3u, dist = (pk >> 17) + 1u;
  const uint32_t e = p - dist + (len < dist ? len : dist);
  return (uint64_t)p | (uint64_t)len << 16 | (uint64_t)dist << 32 | (uint64_t)e << 48;
}

// One wave per workgroup: LDS operations of a wave execute in issue order, so ordering the
// lanes' LDS accesses needs no s_barrier, only that the compiler keep program order across
// lanes (a workgroup fence + wave barrier).
__device__ __forceinline__ void rs_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  __builtin_amdgcn_wave_barrier();
}
// Between the phases of a dataflow round only program order matters: a wave's LDS
// instructions execute in issue order, so a compiler barrier is enough (no lgkmcnt drain).
__device__ __forceinline__ void rs_lds_order() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// set / clear bits [x, x + n) of an LDS bitmap (other lanes touch the same words: atomics)
__device__ __forceinline__ void rs_bits(uint32_t* bm, uint32_t x, uint32_t n, bool set) {
  uint32_t w = x >> 5, o = x & 31u;
  while (n) {
    const uint32_t k = n < 32u - o ? n : 32u - o;
    const uint32_t m = (k == 32u ? ~0u : ((1u << k) - 1u)) << o;
    if (set) atomicOr(bm + w, m);
    else atomicAnd(bm + w, ~m);
    n -= k;
    ++w;
    o = 0;
  }
}
// any bit of [x, y) set
__device__ __forceinline__ bool rs_any_bit(const uint32_t* bm, uint32_t x, uint32_t y) {
  uint32_t w = x >> 5, o = x & 31u;
  uint32_t n = y - x;
  while (n) {
    const uint32_t k = n < 32u - o ? n : 32u - o;
    const uint32_t m = (k == 32u ? ~0u : ((1u << k) - 1u)) << o;
    if (bm[w] & m) return true;
    n -= k;
    ++w;
    o = 0;
  }
  return false;
}

__device__ __forceinline__ uint64_t lds_rd64(const uint8_t* p) { return *(const uint64_t*)p; }

// write the low n (1..8) bytes of v at p
__device__ __forceinline__ void lds_wr_part(uint8_t* p, uint64_t v, uint32_t n) {
  if (n >= 8) {
    *(uint64_t*)p = v;
    return;
  }
  if (n & 4u) {
    *(uint32_t*)p = (uint32_t)v;
    p += 4;
    v >>= 32;
  }
  if (n & 2u) {
    *(uint16_t*)p = (uint16_t)v;
    p += 2;
    v >>= 16;
  }
  if (n & 1u) *p = (uint8_t)v;
}

// 8 bytes of the period-d (1..7) sequence whose first d bytes are the low bytes of v
__device__ __forceinline__ uint64_t periodic8(uint64_t v, uint64_t sel) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  const uint32_t r0 = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel);
  const uint32_t r1 = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
  return (uint64_t)r0 | (uint64_t)r1 << 32;
}

// 4 bytes at any LDS index x from two dword-aligned reads (a byte-aligned ds_read_b32 replays)
__device__ __forceinline__ uint32_t lds_rd32u(const uint8_t* buf, uint32_t x) {
  const uint32_t a = x & ~3u;
  return __builtin_amdgcn_alignbit(*(const uint32_t*)(buf + a + 4u), *(const uint32_t*)(buf + a), (x & 3u) * 8u);
}

// LZ77 copy inside the LDS window: dst index di, len bytes from di - dist (sources final).
__device__ __forceinline__ void rs_copy_lds(uint8_t* __restrict__ buf, uint32_t di, uint32_t len,
                                            uint32_t dist, const uint64_t* __restrict__ s_sel) {
  uint8_t* d = buf + di;
  const uint8_t* s = buf + (di - dist);
  if (dist < 8u) {
    // period < 8: one 8-byte pattern, stamped every cs = d*floor(8/d) bytes
    const uint64_t pat = periodic8(lds_rd64(s), s_sel[dist]);
    const uint32_t cs = (dist == 3u || dist == 6u) ? 6u : (dist == 5u) ? 5u : (dist == 7u) ? 7u : 8u;
    uint32_t t = 0;
    for (; t + 8u <= len; t += cs) *(uint64_t*)(d + t) = pat;
    if (t < len) lds_wr_part(d + t, pat, len - t);
  } else if (dist >= len || dist >= 32u) {
    // 32-byte groups: a group's sources lie before its destination
    for (uint32_t t = 0; t < len; t += 32u) {
      // 16-byte reads (an unaligned ds_read2_b64 pair is not used)
      const uint4 q0 = *(const uint4*)(s + t), q1 = *(const uint4*)(s + t + 16);
      const uint64_t v0 = q0.x | (uint64_t)q0.y << 32, v1 = q0.z | (uint64_t)q0.w << 32,
                     v2 = q1.x | (uint64_t)q1.y << 32, v3 = q1.z | (uint64_t)q1.w << 32;
      const uint32_t n = len - t;
      lds_wr_part(d + t, v0, n);
      if (n > 8u) lds_wr_part(d + t + 8, v1, n - 8u);
      if (n > 16u) lds_wr_part(d + t + 16, v2, n - 16u);
      if (n > 24u) lds_wr_part(d + t + 24, v3, n - 24u);
    }
  } else {
    // 8 <= dist < 32, overlapping: 8-byte chunks in order
    for (uint32_t t = 0; t < len; t += 8u) lds_wr_part(d + t, lds_rd64(s + t), len - t);
  }
}

// copy len bytes from final global bytes g (dist > len) into the LDS window at index di
__device__ __forceinline__ void rs_copy_glb(uint8_t* __restrict__ buf, uint32_t di, uint32_t len,
                                            const uint8_t* __restrict__ g) {
  uint8_t* d = buf + di;
  for (uint32_t t = 0; t < len; t += 32u) {
    // byte-aligned 8-byte global loads (the device runs in unaligned access mode)
    // (requesting only the words a match covers, as exec-masked loads, ran slower: 21.45 ->
    // 22.2 ms at 5 GB, profiles/r03/ab/resolve_condld_5g.txt)
    // (as two 16-byte loads: 21.34 vs 21.39 ms at 5 GB, no gain;
    // profiles/r03/ab/decode_fixed_hoist_and_resolve_g16_5g.txt)
    const uint64_t v0 = *(const uint64_t*)(g + t), v1 = *(const uint64_t*)(g + t + 8),
                   v2 = *(const uint64_t*)(g + t + 16), v3 = *(const uint64_t*)(g + t + 24);
    const uint32_t n = len - t;
    lds_wr_part(d + t, v0, n);
    if (n > 8u) lds_wr_part(d + t + 8, v1, n - 8u);
    if (n > 16u) lds_wr_part(d + t + 16, v2, n - 16u);
    if (n > 24u) lds_wr_part(d + t + 24, v3, n - 24u);
  }
}


__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x, uint32_t lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_up(x, off);
    if ((int)lane >= off) x += t;
  }
  return x;
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {  // set bits below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

}  // namespace hbam
