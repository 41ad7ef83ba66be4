// Micro-benchmark: random 4-byte dictionary gathers on gfx950, from global
// memory (L1/L2) and from an LDS-resident copy, per dictionary bit width.
// Each lane gathers G keys (a hash of its index) and stores the values as
// the decode kernel would (16 contiguous bytes per lane per row).
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_bench.hip -o /tmp/gb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; return x;
}

// one wave per 2048 values: 8 rows of 256 (4 per lane)
__global__ __launch_bounds__(256) void g_global(const uint32_t *dict, uint32_t mask, uint32_t *out, int n) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int v0 = wave * 2048;
  if (v0 >= n) return;
  uint32_t val[8][4];
#pragma unroll
  for (int r = 0; r < 8; r++)
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t k = hsh(v0 + r * 256 + 4 * lane + q) & mask;
      val[r][q] = dict[k];
    }
#pragma unroll
  for (int r = 0; r < 8; r++) {
    uint4 *o = (uint4 *)(out + v0 + r * 256) + lane;
    *o = make_uint4(val[r][0], val[r][1], val[r][2], val[r][3]);
  }
}

// persistent: a workgroup of 1024 threads copies the dictionary into LDS once,
// then its 16 waves take 2048-value jobs round-robin
__global__ __launch_bounds__(1024) void g_lds(const uint32_t *dict, uint32_t dn, uint32_t mask, uint32_t *out, int n, int nwg) {
  extern __shared__ uint32_t sd[];
  for (uint32_t i = threadIdx.x; i < dn; i += 1024) sd[i] = dict[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  for (int job = blockIdx.x * 16 + wv; job * 2048 < n; job += nwg * 16) {
    const int v0 = job * 2048;
    uint32_t val[8][4];
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t k = hsh(v0 + r * 256 + 4 * lane + q) & mask;
        val[r][q] = sd[k];
      }
#pragma unroll
    for (int r = 0; r < 8; r++) {
      uint4 *o = (uint4 *)(out + v0 + r * 256) + lane;
      *o = make_uint4(val[r][0], val[r][1], val[r][2], val[r][3]);
    }
  }
}

// keys only (no gather): the hash + store skeleton
__global__ __launch_bounds__(256) void g_none(uint32_t mask, uint32_t *out, int n) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int v0 = wave * 2048;
  if (v0 >= n) return;
#pragma unroll
  for (int r = 0; r < 8; r++) {
    uint32_t v[4];
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = hsh(v0 + r * 256 + 4 * lane + q) & mask;
    uint4 *o = (uint4 *)(out + v0 + r * 256) + lane;
    *o = make_uint4(v[0], v[1], v[2], v[3]);
  }
}

int main() {
  const int n = 1 << 26;  // 64M values, 256 MB out
  uint32_t *dict, *out;
  CK(hipMalloc(&dict, (1u << 22) * 4));
  CK(hipMalloc(&out, (size_t)n * 4));
  std::vector<uint32_t> h(1u << 22);
  for (size_t i = 0; i < h.size(); i++) h[i] = (uint32_t)(i * 2654435761u);
  CK(hipMemcpy(dict, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = n / 2048 / 4;
  CK(hipFuncSetAttribute((const void *)g_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  int cus = 256;
  auto timeit = [&](auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int i = 0; i < 10; i++) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 10;
  };
  {
    const float ms = timeit([&] { hipLaunchKernelGGL(g_none, grid, 256, 0, 0, 0xffu, out, n); });
    printf("none        %7.3f ms  %6.1f Gval/s  %6.0f GB/s out\n", ms, n / ms / 1e6, n * 4.0 / ms / 1e6);
  }
  for (int bw = 2; bw <= 22; bw += 1) {
    const uint32_t mask = (1u << bw) - 1;
    const float mg = timeit([&] { hipLaunchKernelGGL(g_global, grid, 256, 0, 0, dict, mask, out, n); });
    float ml = -1;
    if (bw <= 15) {
      const uint32_t dn = 1u << bw;
      int nwg = cus * (dn * 4 <= 80 * 1024 ? 2 : 1);
      if (dn * 4 <= 40 * 1024) nwg = cus * 4;
      if (dn * 4 <= 20 * 1024) nwg = cus * 8 > cus * 4 ? cus * 4 : cus * 4;
      ml = timeit([&] { hipLaunchKernelGGL(g_lds, nwg, 1024, dn * 4, 0, dict, dn, mask, out, n, nwg); });
    }
    printf("bw %2d global %7.3f ms %6.1f Gval/s | lds %7.3f ms %6.1f Gval/s\n", bw, mg, n / mg / 1e6, ml,
           ml > 0 ? n / ml / 1e6 : 0.0);
  }
  return 0;
}
