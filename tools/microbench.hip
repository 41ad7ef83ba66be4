// microbench.hip — copy-pattern microbenchmarks used to size the Snappy and
// decode kernels (not part of the product).  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

// (a) plain aligned streaming copy, 16 B per lane, grid-stride
__global__ void k_copy_aligned(const uint4 *__restrict__ s, uint4 *__restrict__ d, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

// (b) one wave per "page", page-sized chunk copied with skewed source like copy_literal
template <bool GLOBAL>
__global__ void k_copy_wave(const uint8_t *s, uint8_t *d, int64_t page, int npages, int skew) {
  int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (wave >= npages) return;
  const uint8_t *S = s + (int64_t)wave * page + skew;
  uint8_t *D = d + (int64_t)wave * page;
  const uint32_t sk = (uint32_t)((uintptr_t)S & 3);
  const uint32_t *SA = (const uint32_t *)((uintptr_t)S & ~(uintptr_t)3);
  int64_t body = page / 16 - 1;
  for (int64_t c = lane; c < body; c += 128) {
    int64_t c2 = c + 64;
    uint4 a, b = make_uint4(0, 0, 0, 0);
    uint32_t a4, b4 = 0;
    if (GLOBAL) {
      typedef __attribute__((address_space(1))) const uint32_t gu32;
      gu32 *g = (gu32 *)(SA + 4 * c);
      a.x = g[0]; a.y = g[1]; a.z = g[2]; a.w = g[3];
      a4 = g[4];
    } else {
      a = *(const uint4 *)(SA + 4 * c);
      a4 = SA[4 * c + 4];
    }
    if (c2 < body) {
      b = *(const uint4 *)(SA + 4 * c2);
      b4 = SA[4 * c2 + 4];
    }
    uint4 o;
    o.x = __builtin_amdgcn_alignbyte(a.y, a.x, sk);
    o.y = __builtin_amdgcn_alignbyte(a.z, a.y, sk);
    o.z = __builtin_amdgcn_alignbyte(a.w, a.z, sk);
    o.w = __builtin_amdgcn_alignbyte(a4, a.w, sk);
    *(uint4 *)(D + 16 * c) = o;
    if (c2 < body) {
      uint4 p;
      p.x = __builtin_amdgcn_alignbyte(b.y, b.x, sk);
      p.y = __builtin_amdgcn_alignbyte(b.z, b.y, sk);
      p.z = __builtin_amdgcn_alignbyte(b.w, b.z, sk);
      p.w = __builtin_amdgcn_alignbyte(b4, b.w, sk);
      *(uint4 *)(D + 16 * c2) = p;
    }
  }
}

// (c) gather: out[i] = dict[idx[i]] for a random index stream
__global__ void k_gather(const uint32_t *__restrict__ idx, const uint32_t *__restrict__ dict, uint32_t *__restrict__ out,
                         size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = dict[idx[i]];
}

int main() {
  const size_t N = 160ull << 20;
  uint8_t *a, *b;
  hipMalloc(&a, N + 4096);
  hipMalloc(&b, N + 4096);
  hipMemset(a, 1, N);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms;
  for (int rep = 0; rep < 2; rep++) {
    hipEventRecord(e0);
    k_copy_aligned<<<2048, 256>>>((const uint4 *)a, (uint4 *)b, N / 16);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("aligned grid copy %zu MB: %.3f ms = %.0f GB/s (r+w)\n", N >> 20, ms, 2.0 * N / ms / 1e6);
  }
  for (int64_t page : {4096L, 32768L, 65536L}) {
    int np = (int)(N / page) - 1;
    for (int skew : {0, 1}) {
      for (int g = 0; g < 2; g++) {
        hipEventRecord(e0);
        if (g) k_copy_wave<true><<<(np + 3) / 4, 256>>>(a, b, page, np, skew);
        else k_copy_wave<false><<<(np + 3) / 4, 256>>>(a, b, page, np, skew);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("wave-per-page copy page=%lld skew=%d %s: %.3f ms = %.0f GB/s (r+w)\n", (long long)page, skew,
               g ? "global" : "flat", ms, 2.0 * np * page / ms / 1e6);
      }
    }
  }
  // gather
  size_t n = 100ull << 20;
  uint32_t *idx, *dict, *out;
  hipMalloc(&idx, n * 4);
  hipMalloc(&out, n * 4);
  hipMalloc(&dict, (1 << 20) * 4);
  uint32_t *h = (uint32_t *)malloc(n * 4);
  uint64_t x = 88172645463325252ull;
  for (size_t i = 0; i < n; i++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    h[i] = (uint32_t)(x & ((1 << 20) - 1));
  }
  hipMemcpy(idx, h, n * 4, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; rep++) {
    hipEventRecord(e0);
    k_gather<<<4096, 256>>>(idx, dict, out, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("gather 100M from 4MB dict: %.3f ms = %.0f GB/s (idx+out)\n", ms, 8.0 * n / ms / 1e6);
  }
  return 0;
}
