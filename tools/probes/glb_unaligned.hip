// Probe: unaligned global_load_dwordx2 / dwordx4 and global_store_dwordx2 at byte offsets.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k(const uint8_t* src, uint64_t* out, uint8_t* wbuf) {
  const uint32_t l = threadIdx.x;
  out[l] = *(const uint64_t*)(src + l + 1);
  const uint4 q = *(const uint4*)(src + 100 + l);
  out[64 + l] = q.x | (uint64_t)q.y << 32;
  out[128 + l] = q.z | (uint64_t)q.w << 32;
  if (l < 40) *(uint64_t*)(wbuf + 9 * l + 3) = 0x0102030405060708ULL * (l + 1);
}

int main() {
  uint8_t h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = (uint8_t)(i * 13 + 5);
  uint8_t *d, *w;
  uint64_t* o;
  if (hipMalloc(&d, 1024) || hipMalloc(&o, 192 * 8) || hipMalloc(&w, 1024)) return 2;
  if (hipMemcpy(d, h, 1024, hipMemcpyHostToDevice) || hipMemset(w, 0, 1024)) return 2;
  k<<<1, 64>>>(d, o, w);
  uint64_t ho[192];
  uint8_t hw[1024];
  if (hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost) || hipMemcpy(hw, w, 1024, hipMemcpyDeviceToHost)) return 2;
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    uint64_t e, e1, e2;
    __builtin_memcpy(&e, h + l + 1, 8);
    __builtin_memcpy(&e1, h + 100 + l, 8);
    __builtin_memcpy(&e2, h + 108 + l, 8);
    if (ho[l] != e || ho[64 + l] != e1 || ho[128 + l] != e2) ++bad;
  }
  uint8_t ew[1024] = {0};
  for (int l = 0; l < 40; ++l) { uint64_t v = 0x0102030405060708ULL * (l + 1); __builtin_memcpy(ew + 9 * l + 3, &v, 8); }
  for (int i = 0; i < 1024; ++i) bad += ew[i] != hw[i];
  printf("unaligned global probe: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
  return bad != 0;
}
