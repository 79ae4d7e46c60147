// Probe: do unaligned ds_read_b64/b128 and ds_write_b64/b32 work on this device?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k(uint64_t* out, uint32_t* out2) {
  __shared__ __attribute__((aligned(16))) uint8_t s[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) s[i] = (uint8_t)(i * 7 + 3);
  __syncthreads();
  const uint32_t off = threadIdx.x;  // unaligned for most lanes
  uint64_t v = *(const uint64_t*)(s + off);
  uint4 q = *(const uint4*)(s + 256 + off);
  out[threadIdx.x] = v;
  out[64 + threadIdx.x] = ((uint64_t)q.y << 32) | q.x;
  out[128 + threadIdx.x] = ((uint64_t)q.w << 32) | q.z;
  __syncthreads();
  // unaligned writes: lane l writes 8 bytes at 600 + 9*l (disjoint)
  if (threadIdx.x < 40) *(uint64_t*)(s + 512 + 9 * threadIdx.x + 1) = 0x1122334455667788ULL + threadIdx.x;
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += 64) ((uint8_t*)out2)[i] = s[i];
}

int main() {
  uint64_t* d; uint32_t* d2;
  hipMalloc(&d, 192 * 8); hipMalloc(&d2, 1024);
  k<<<1, 64>>>(d, d2);
  uint64_t h[192]; uint8_t h2[1024];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  hipMemcpy(h2, d2, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  uint8_t s[1024];
  for (int i = 0; i < 1024; ++i) s[i] = (uint8_t)(i * 7 + 3);
  for (int l = 0; l < 64; ++l) {
    uint64_t e; __builtin_memcpy(&e, s + l, 8);
    uint64_t e1, e2; __builtin_memcpy(&e1, s + 256 + l, 8); __builtin_memcpy(&e2, s + 264 + l, 8);
    if (h[l] != e || h[64 + l] != e1 || h[128 + l] != e2) { if (bad < 5) printf("read mismatch lane %d\n", l); ++bad; }
  }
  for (int l = 0; l < 40; ++l) { uint64_t v = 0x1122334455667788ULL + l; __builtin_memcpy(s + 512 + 9 * l + 1, &v, 8); }
  for (int i = 0; i < 1024; ++i) if (s[i] != h2[i]) { if (bad < 10) printf("write mismatch at %d\n", i); ++bad; }
  printf("unaligned LDS probe: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
  return bad != 0;
}
