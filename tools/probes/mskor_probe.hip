// ds_mskor_b32 semantics probe (k_resolve_units relies on D = (D & ~DATA0) | DATA1): 64 lanes
// write disjoint bytes of 16 shared dwords in one instruction; prints PASS/FAIL.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned* out) {
  __shared__ unsigned s[16];
  const unsigned l = threadIdx.x;
  if (l < 16) s[l] = 0x11223344u;
  __syncthreads();
  const unsigned addr = (unsigned)(uintptr_t)(s + (l >> 2)), b = l & 3u;
  const unsigned m = 0xffu << (8u * b), v = ((0xa0u + l) & 0xffu) << (8u * b);
  asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(addr), "v"(m), "v"(v) : "memory");
  __syncthreads();
  if (l < 16) out[l] = s[l];
}

int main() {
  unsigned* d;
  unsigned h[16];
  if (hipMalloc(&d, 64) != hipSuccess) return 2;
  k<<<1, 64>>>(d);
  if (hipMemcpy(h, d, 64, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int bad = 0;
  for (unsigned w = 0; w < 16; ++w) {
    unsigned want = 0;
    for (unsigned b = 0; b < 4; ++b) want |= ((0xa0u + 4 * w + b) & 0xffu) << (8 * b);
    if (h[w] != want) {
      printf("dword %u: got %08x want %08x\n", w, h[w], want);
      ++bad;
    }
  }
  printf(bad ? "FAIL\n" : "PASS ds_mskor_b32 = (D & ~data0) | data1, concurrent bytes kept\n");
  return bad ? 1 : 0;
}
