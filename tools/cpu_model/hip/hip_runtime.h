// CPU model build of the Huffman pass (tools/cpu_model): the few HIP names inflate_dev.h /
// inflate_tok.h use, for a host compile of ONE lane's decode under MemorySanitizer.  Diagnostic
// only — nothing in the product links this; the GPU build uses the real <hip/hip_runtime.h>.
#pragma once
#include <stdint.h>
#include <string.h>

#define __device__
#define __host__
#define __global__
#define __forceinline__ inline __attribute__((always_inline))

struct uint4 {
  uint32_t x, y, z, w;
};
static inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
  uint4 v;
  v.x = x;
  v.y = y;
  v.z = z;
  v.w = w;
  return v;
}

// one lane: the first active lane is this lane; waits and clocks are no-ops
#define __builtin_amdgcn_readfirstlane(x) (x)
#define __builtin_amdgcn_ballot_w64(x) ((uint64_t)((x) ? 1u : 0u))
#define __builtin_amdgcn_s_waitcnt(x) ((void)0)
#define __builtin_amdgcn_s_memtime() ((uint64_t)0)
