// resolve_dev.h — LZ77 resolution (phase 2 of the batched inflate): the contract and the shared
// stretch geometry; the kernel is k_resolve_units (resolve_units.h), one wave per BGZF block.
//
// Input (left in ubuf by k_inflate_tokens): literals at their final offsets, a 3-byte
// descriptor (len-3, dist-1 as u8 + u16 LE) at the first bytes of every match of >= 3 bytes,
// one bit per match start in the block's bitmap, and an optional final match of < 3 bytes
// (`tails`).  Output: the block's inflated bytes, in place.
//
// The block is walked in stretches of RS_S output bytes.  LDS holds a window of the RS_W
// bytes before the stretch, the stretch and the next stretch (matches spill up to 258 bytes
// past their stretch), ~4.9 KiB per wave with the unit list: 8 waves per SIMD.  Per stretch:
//   1. the stretch's match starts come from 32 bitmap words (one per lane), their descriptors
//      are read once and cut into <= 16-byte units, split into
//        - "pre" units (their match's source ends before the stretch: every source byte is
//          final), copied all at once, from the LDS window or (older than the window, already
//          written back) from ubuf;
//        - "ordered" units (source inside the stretch, or a periodic match), executed in
//          dataflow rounds: a unit runs once no earlier unit still has to write its source;
//   2. the stretch is written back to ubuf and the window slides by RS_S.
// The raw bytes of stretch k+2 are requested after stretch k's pre units, its bitmap words
// before stretch k-1's drain.
#pragma once
#include <stdint.h>

namespace hbam {

// window kept in LDS behind the stretch.  A/B at 2 GB (stretch 2 KiB): 4096 -> 20.0 ms, 2048 ->
// 18.0, 1024 -> 16.7; at 10 GB with packed match records and 8 waves/SIMD: 1024 -> 48.8 ms (LDS
// caps it at 7 waves), 512 -> 42.6 ms (profiles/r02/s2/ab_resolve_occupancy_10g.txt); with the
// units kernel at 5 GB: 512 15.4, 1 KiB 16.3, 2 KiB 17.0 ms (profiles/r05/ab/resolve_window_*)
constexpr uint32_t RS_W = 512;
// stretch (output bytes).  A/B at 2 GB (window 1 KiB): 2048 -> 16.8 ms, 1024 -> 11.7 ms;
// k_resolve_units' unit records need 1 KiB
constexpr uint32_t RS_S = 1024;
constexpr uint32_t RS_C = RS_S / 1024;                // 16-byte columns per lane per stretch
constexpr uint32_t RS_BUF = RS_W + 2 * RS_S + 48;     // + pad for 32-byte over-reads
static_assert(RS_W >= 16 && RS_W % 16 == 0 && (RS_S == 1024 || RS_S == 2048),
              "window: whole 16-byte columns; stretch: 1 or 2 KiB (one or two columns per lane)");
constexpr uint32_t RS_MAXM = RS_S / 3 + 2;            // matches starting in one stretch
constexpr uint32_t RS_PW = (RS_S + 16 + 258 + 31) / 32 + 1;  // pending-byte words of a stretch + spill


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

// 4 bytes at any LDS index x from two dword-aligned reads (a byte-aligned ds_read_b32 replays)
__device__ __forceinline__ uint32_t lds_rd32u(const uint8_t* buf, uint32_t x) {
  const uint32_t a = x & ~3u;
  return __builtin_amdgcn_alignbit(*(const uint32_t*)(buf + a + 4u), *(const uint32_t*)(buf + a), (x & 3u) * 8u);
}

__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x, uint32_t lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_up(x, off);
    if ((int)lane >= off) x += t;
  }
  return x;
}

// inclusive wave scan (+) with DPP row shifts and row broadcasts (GFX9 DPP): no LDS traffic, where
// a __shfl_up scan is six ds_bpermute_b32 through the LDS pipe
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}
__device__ __forceinline__ uint32_t wave_last(uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 63); }

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {  // set bits below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

}  // namespace hbam
