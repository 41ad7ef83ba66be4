// Micro-benchmark (analysis only): what bounds random 4-byte dictionary
// gathers from dictionaries past the L1 (256 KiB .. 4 MiB, C2's bit widths
// 16-20) on gfx950, by load cache policy, and what an LDS-resident part of the
// dictionary buys.  Each lane gathers 4 keys a row (a hash of the value
// index), 8 rows a wave (2048 values, one k_expand job), all 32 gathers in
// flight, then 16-byte stores, as k_expand_mix does.
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_bench2.hip -o /tmp/gb2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}

// AUX: buffer-load cache policy bits (gfx950: 1 = sc0, 2 = nt, 16 = sc1)
template <int AUX>
__global__ __launch_bounds__(256) void g_buf(const uint32_t *dict, uint32_t dn, uint32_t *out, int n) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int v0 = wave * 2048;
  if (v0 >= n) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)dict, (short)0, (int)(dn * 4), 0x00020000);
  uint32_t val[8][4];
#pragma unroll
  for (int r = 0; r < 8; r++)
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t k = hsh(v0 + r * 256 + 4 * lane + q) % dn;
      val[r][q] = __builtin_amdgcn_raw_buffer_load_b32(rs, k * 4, 0, AUX);
    }
#pragma unroll
  for (int r = 0; r < 8; r++) {
    uint4 *o = (uint4 *)(out + v0 + r * 256) + lane;
    *o = make_uint4(val[r][0], val[r][1], val[r][2], val[r][3]);
  }
}

// the first `pn` entries of the dictionary resident in LDS (one 1024-thread
// workgroup a CU, persistent), the rest gathered from L1/L2
__global__ __launch_bounds__(1024) void g_part(const uint32_t *dict, uint32_t dn, uint32_t pn, uint32_t *out, int n, int nwg) {
  extern __shared__ uint32_t sd[];
  for (uint32_t i = threadIdx.x; i < pn; i += 1024) sd[i] = dict[i];
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)dict, (short)0, (int)(dn * 4), 0x00020000);
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  for (int job = blockIdx.x * 16 + wv; job * 2048 < n; job += nwg * 16) {
    const int v0 = job * 2048;
    uint32_t val[8][4];
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t k = hsh(v0 + r * 256 + 4 * lane + q) % dn;
        val[r][q] = k < pn ? sd[k] : __builtin_amdgcn_raw_buffer_load_b32(rs, k * 4, 0, 0);
      }
#pragma unroll
    for (int r = 0; r < 8; r++) {
      uint4 *o = (uint4 *)(out + v0 + r * 256) + lane;
      *o = make_uint4(val[r][0], val[r][1], val[r][2], val[r][3]);
    }
  }
}

// multi-pass: the dictionary streamed through LDS in slices of `sn` entries;
// 16 waves each hold one job's keys in registers (2048 values a wave), every
// slice gathers the keys inside it
__global__ __launch_bounds__(1024) void g_pass(const uint32_t *dict, uint32_t dn, uint32_t sn, uint32_t *out, int n, int nwg) {
  extern __shared__ uint32_t sd[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  for (int grp = blockIdx.x; grp * 16 * 2048 < n; grp += nwg) {
    const int v0 = (grp * 16 + wv) * 2048;
    uint32_t key[8][4], val[8][4];
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        key[r][q] = hsh(v0 + r * 256 + 4 * lane + q) % dn;
        val[r][q] = 0;
      }
    for (uint32_t base = 0; base < dn; base += sn) {
      __syncthreads();
      const uint32_t m = min(sn, dn - base);
      for (uint32_t i = threadIdx.x * 4; i < m; i += 4096) *(uint4 *)(sd + i) = *(const uint4 *)(dict + base + i);
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 8; r++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint32_t rel = key[r][q] - base;
          if (rel < m) val[r][q] = sd[rel];
        }
    }
    if (v0 < n) {
#pragma unroll
      for (int r = 0; r < 8; r++) {
        uint4 *o = (uint4 *)(out + v0 + r * 256) + lane;
        *o = make_uint4(val[r][0], val[r][1], val[r][2], val[r][3]);
      }
    }
  }
}

int main() {
  const int n = 1 << 25;  // 32M values, 128 MB out
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
  CK(hipFuncSetAttribute((const void *)g_part, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void *)g_pass, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  auto timeit = [&](auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int i = 0; i < 10; i++) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return n / (ms / 10) / 1e6;  // Gvalues/s
  };
  printf("dict entries: Gval/s  plain  sc0  nt  sc1 sc0+sc1 | part-LDS 128K | pass 32K-entry slices\n");
  for (int bw = 13; bw <= 21; bw++) {
    const uint32_t dn = (bw == 21) ? 700000u : (1u << bw);
    const float p0 = timeit([&] { hipLaunchKernelGGL(g_buf<0>, grid, 256, 0, 0, dict, dn, out, n); });
    const float p1 = timeit([&] { hipLaunchKernelGGL(g_buf<1>, grid, 256, 0, 0, dict, dn, out, n); });
    const float p2 = timeit([&] { hipLaunchKernelGGL(g_buf<2>, grid, 256, 0, 0, dict, dn, out, n); });
    const float p3 = timeit([&] { hipLaunchKernelGGL(g_buf<16>, grid, 256, 0, 0, dict, dn, out, n); });
    const float p4 = timeit([&] { hipLaunchKernelGGL(g_buf<17>, grid, 256, 0, 0, dict, dn, out, n); });
    const uint32_t pn = dn < 32768 ? dn : 32768;
    const float pl = timeit([&] { hipLaunchKernelGGL(g_part, 256, 1024, pn * 4, 0, dict, dn, pn, out, n, 256); });
    const float ps = timeit([&] { hipLaunchKernelGGL(g_pass, 256, 1024, 32768 * 4, 0, dict, dn, 32768u, out, n, 256); });
    printf("%8u: %6.0f %6.0f %6.0f %6.0f %6.0f | %6.0f | %6.0f\n", dn, p0, p1, p2, p3, p4, pl, ps);
  }
  return 0;
}
