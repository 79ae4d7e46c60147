// Probe: cost of LDS accesses at byte offsets off their natural alignment, for the access kinds
// k_resolve uses (8-byte reads/writes at match offsets, 16-byte reads, 4-/2-byte pieces).  The
// guide (cdna_hip_programming.md, Guideline 17) states _b64/_b128 accesses off 8/16-byte alignment
// replay at 64 cycles per wave-instruction; this measures each kind aligned vs misaligned.
// Prints one line per kind: ns per wave-instruction (whole-chip throughput, 8 waves per CU).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ITERS = 4096;

template <int KIND>
__global__ __launch_bounds__(64) void k(uint32_t shift, uint64_t* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t s[4096 + 64];
  for (int i = threadIdx.x; i < 4096 + 64; i += 64) s[i] = (uint8_t)i;
  __syncthreads();
  const uint32_t lane = threadIdx.x;
  uint64_t acc = 0;
  uint32_t base = lane * 48 + shift;  // lanes 48 B apart: no two lanes share a word
  for (int it = 0; it < ITERS; ++it) {
    const uint32_t a = (base + (it & 7) * 16) & 4095;
    uint8_t* p = s + a;
    if (KIND == 0) acc += *(const uint64_t*)p;                       // ds_read_b64
    if (KIND == 1) { const uint4 q = *(const uint4*)p; acc += q.x ^ q.w; }  // ds_read_b128
    if (KIND == 2) acc += *(const uint32_t*)p;                       // ds_read_b32
    if (KIND == 3) *(uint64_t*)p = acc + it;                         // ds_write_b64
    if (KIND == 4) *(uint32_t*)p = (uint32_t)acc + it;               // ds_write_b32
    if (KIND == 5) *(uint16_t*)p = (uint16_t)(acc + it);             // ds_write_b16
    if (KIND == 6) acc += p[0];                                      // ds_read_u8
    __builtin_amdgcn_s_waitcnt(0);
  }
  if (acc == 0x123456789ull) sink[0] = acc;
}

template <int KIND>
float run(uint32_t shift, uint64_t* sink) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k<KIND><<<256 * 8, 64>>>(shift, sink);
  hipEventRecord(a);
  k<KIND><<<256 * 8, 64>>>(shift, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  uint64_t* sink;
  hipMalloc(&sink, 64);
  const char* names[] = {"ds_read_b64", "ds_read_b128", "ds_read_b32", "ds_write_b64", "ds_write_b32",
                         "ds_write_b16", "ds_read_u8"};
  const double ops = 256.0 * 8 * ITERS;  // wave-instructions per launch
  for (uint32_t sh : {0u, 1u, 2u, 4u, 8u}) {
    float t[7] = {run<0>(sh, sink), run<1>(sh, sink), run<2>(sh, sink), run<3>(sh, sink),
                  run<4>(sh, sink), run<5>(sh, sink), run<6>(sh, sink)};
    for (int q = 0; q < 7; ++q)
      printf("%-13s offset %%16 = %2u: %.3f ms, %.3f ns per wave-instruction (chip)\n", names[q], sh, t[q],
             t[q] * 1e6 / ops);
  }
  hipFree(sink);
  return 0;
}
