// Checks the lane -> LDS placement of global_load_lds_dwordx4 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k(const uint32_t *src, uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint32_t buf[2048];
  for (int i = threadIdx.x; i < 2048; i += 64) buf[i] = 0xdeadbeef;
  __syncthreads();
  // lane l loads 16 bytes from src + 4 * (63 - l) (reversed), chunk 1 at +1024 B
  __builtin_amdgcn_global_load_lds((const void *)(src + 4 * (63 - threadIdx.x)),
                                   (__attribute__((address_space(3))) void *)buf, 16, 0, 0);
  __builtin_amdgcn_global_load_lds((const void *)(src + 256 + 4 * threadIdx.x),
                                   (__attribute__((address_space(3))) void *)(buf + 256), 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 64) out[i] = buf[i];
}
int main() {
  std::vector<uint32_t> h(1024);
  for (int i = 0; i < 1024; i++) h[i] = i;
  uint32_t *d, *o;
  hipMalloc(&d, 4096);
  hipMalloc(&o, 4096);
  hipMemcpy(d, h.data(), 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  std::vector<uint32_t> r(512);
  hipMemcpy(r.data(), o, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; l++)
    for (int c = 0; c < 4; c++) {
      if (r[4 * l + c] != (uint32_t)(4 * (63 - l) + c)) bad++;
      if (r[256 + 4 * l + c] != (uint32_t)(256 + 4 * l + c)) bad++;
    }
  printf("lds dma placement %s (bad %d) r[0..7]=%u %u %u %u %u %u %u %u\n", bad ? "MISMATCH" : "ok", bad, r[0], r[1],
         r[2], r[3], r[4], r[5], r[256], r[257]);
  return bad != 0;
}
