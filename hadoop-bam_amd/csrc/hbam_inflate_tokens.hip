// hbam_inflate_tokens.hip — k_inflate_tokens, the Huffman lane pass of the batched BGZF inflate
// (inflate_tok.h; replaces [htsjdk] BlockGunzipper.unzipBlock's Inflater on the BAM read path).
//
// Its own translation unit in the product build (__graft_entry__.build(): compiled with
// `-mllvm -amdgpu-sched-strategy=max-ilp` and linked into libhbam.so next to hbam_capi.hip, which
// is compiled with -DHBAM_SPLIT_TOK and only declares the kernel).  The pass runs at two waves per SIMD (its LDS tables
// and registers allow no more) and a wave alone issues at most one instruction per four cycles, so
// the order of its own instructions decides how much of each dependency latency it sits out: the
// ILP-first schedule gives the kernel 30.26 / 30.35 -> 29.82 / 29.93 ms at 5 GB with the same
// output (profiles/r06/ab/huffman_max_ilp_schedule_5g.txt).  Applied to the whole library the same
// strategy costs the occupancy-bound kernels registers (k_decode_pools 90 -> 105 VGPRs), hence the
// split.  The profiling build (-DHBAM_PROF) and hand-made single-command builds include this file
// from hbam_kernels.hip instead (default scheduling).
#ifndef HBAM_INFLATE_TOKENS_HIP
#define HBAM_INFLATE_TOKENS_HIP
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbam_internal.h"
#include "inflate_dev.h"
#include "inflate_tok.h"

namespace hbam {

static_assert(TOK_LENS_END == LENS_SLOT, "k_inflate_tokens: code-length scratch size");
__global__ __launch_bounds__(INFLATE_WG, 2) void k_inflate_tokens(const uint8_t* __restrict__ comp,
                                                                  const BlockRec* __restrict__ blk,
                                                                  const uint64_t* __restrict__ uoff,
                                                                  uint32_t nblk, uint8_t* __restrict__ ubuf,
                                                                  uint8_t* __restrict__ lens_scratch,
                                                                  uint32_t* __restrict__ bitmap,
                                                                  uint32_t* __restrict__ tails,
                                                                  uint8_t* __restrict__ edges,
                                                                  int32_t* __restrict__ status,
                                                                  const uint32_t* __restrict__ list,
                                                                  const uint32_t* __restrict__ nlist) {
  // 320 B of LDS per lane (u8 lit/len + distance symbols): 20 KiB per workgroup -> 8 per CU
  __shared__ uint8_t s_ll[INFLATE_WG * 288];
  __shared__ uint8_t s_d[INFLATE_WG * 32];
  // list mode: the blocks k_inflate_wave left (list[0 .. *nlist)), else blocks 0 .. nblk
  uint32_t b = blockIdx.x * INFLATE_WG + threadIdx.x;
  if (list) {
    if (b >= *nlist) return;
    b = list[b];
  }
  if (b >= nblk) return;
#ifdef HBAM_PROF
  const uint64_t pr0 = PROF_RT(), pc0 = PROF_CLK();
#endif
  const BlockRec r = blk[b];
  uint32_t produced = 0;
  int32_t st;
  tails[2 * (uint64_t)b] = 0;
  if (r.isize > 65536u) {
    st = INF_OK;  // unsupported here; the runtime reports HBAM_EUNSUPPORTED for it
  } else if (r.clen < 26u) {
    st = INF_DATA;  // Inflater.setInput with a negative length
  } else {
    TSink sink;
    sink.init(ubuf, uoff[b], r.isize, bitmap + (uint64_t)b * BITMAP_WORDS, tails + 2 * (uint64_t)b,
              edges + 32 * (uint64_t)b);
#ifdef HBAM_PROF
    uint64_t pt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pc[4] = {0, 0, 0, 0};
#endif
    // per-lane symbol tables, lane-contiguous (dword-interleaving them across the lanes removes
    // the LDS bank conflicts, 75 % of the pass's LDS cycles, but not time: 33.7 vs 34.3 ms at
    // 5 GB, profiles/r03/ab/huffman_interleaved_symtab_5g.txt; re-measured on the round-6 pass:
    // 30.9 / 30.9 -> 31.0 / 31.2 ms, profiles/r06/ab/huffman_interleaved_symtab_5g.txt)
    uint8_t* const my_ll = s_ll + threadIdx.x * 288;
    uint8_t* const my_d = s_d + threadIdx.x * 32;
    st = inflate_tokens_block(comp + r.coff + 18, r.clen - 26u, r.isize, my_ll, my_d,
                              lens_scratch + (uint64_t)b * LENS_SLOT, sink,
                              &produced
#ifdef HBAM_PROF
                              , pt, pc
#endif
                              );
#ifdef HBAM_PROF
    if (g_prof) {
      for (int q = 0; q < 8; ++q) g_prof[32 * (uint64_t)b + 16 + q] = pt[q];
      for (int q = 0; q < 4; ++q) g_prof[32 * (uint64_t)b + 24 + q] = pc[q];
    }
#endif
  }
  status[b] = st;
#ifdef HBAM_PROF
  if (g_prof) {
    g_prof[32 * (uint64_t)b + 8] = pr0;
    g_prof[32 * (uint64_t)b + 9] = PROF_RT();
    g_prof[32 * (uint64_t)b + 10] = PROF_CLK() - pc0;
    g_prof[32 * (uint64_t)b + 11] = produced;
  }
#endif
}

}  // namespace hbam
#endif  // HBAM_INFLATE_TOKENS_HIP
