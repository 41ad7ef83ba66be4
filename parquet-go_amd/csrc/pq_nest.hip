// pq_nest.hip — the list structure of columns with max_rep >= 2 (Arrow
// List<...List<T>>) from their decoded levels (NestArgs, pq_common.h).
//
// The reference hands such a column back as levels and values
// (ColumnStore.get, data_store.go:158-203: a value's array ends at the first
// rep level below max_rep; the outer levels are rebuilt from rep / def by
// the row reader, schema.go:171-264).  Here every repetition level k gets
// Arrow offsets and a validity bitmap, and the leaf slots a validity bitmap
// that places the dense values (pqg_batch_column_nest).  Two launches over
// blocks of NEST_CH level entries: per-block flag counts, then each block
// scans its entries (ballot / mbcnt within a wave, wave totals through LDS)
// from the counts of the blocks before it.
#include <hip/hip_runtime.h>

#include "pq_common.h"
#include "pq_device.h"

namespace pq {
namespace {

__device__ __forceinline__ uint32_t nest_flags(const NestArgs &a, int64_t i) {
  if (i >= a.n) return 0u;
  const int r = a.rep[i], d = a.def[i];
  uint32_t f = r == 0 ? 1u : 0u;
  for (int k = 1; k <= a.max_rep; k++)
    if (r <= k && d >= a.rdef[k]) f |= 1u << k;
  return f;
}

__global__ __launch_bounds__(256) void k_nest_count(NestArgs a) {
  __shared__ int32_t tot[NEST_MAXR + 1];
  if (threadIdx.x <= NEST_MAXR) tot[threadIdx.x] = 0;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * NEST_CH;
  int32_t c[NEST_MAXR + 1] = {0};
  for (int t = threadIdx.x; t < NEST_CH; t += 256) {
    const uint32_t f = nest_flags(a, lo + t);
#pragma unroll
    for (int j = 0; j <= NEST_MAXR; j++) c[j] += (f >> j) & 1u;
  }
#pragma unroll
  for (int j = 0; j <= NEST_MAXR; j++)
    if (j <= a.max_rep && c[j]) atomicAdd(&tot[j], c[j]);
  __syncthreads();
  if ((int)threadIdx.x <= a.max_rep) a.sums[(int64_t)blockIdx.x * (a.max_rep + 1) + threadIdx.x] = tot[threadIdx.x];
}

__global__ __launch_bounds__(256) void k_nest_write(NestArgs a) {
  __shared__ int64_t base[NEST_MAXR + 1];
  __shared__ int32_t wtot[4][NEST_MAXR + 1];
  const int R = a.max_rep;
  const int lane = lane_id(), w = (int)(threadIdx.x >> 6);
  if ((int)threadIdx.x <= R) base[threadIdx.x] = 0;
  __syncthreads();
  // the counts of the blocks before this one
  {
    int64_t c[NEST_MAXR + 1] = {0};
    for (int b = threadIdx.x; b < (int)blockIdx.x; b += 256)
      for (int j = 0; j <= R; j++) c[j] += a.sums[(int64_t)b * (R + 1) + j];
    for (int j = 0; j <= R; j++)
      if (c[j]) atomicAdd((unsigned long long *)&base[j], (unsigned long long)c[j]);
  }
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * NEST_CH;
  for (int s = 0; s < NEST_CH; s += 256) {
    const int64_t i = lo + s + threadIdx.x;
    const uint32_t f = nest_flags(a, i);
    int32_t pre[NEST_MAXR + 1];
    for (int j = 0; j <= R; j++) {
      const uint64_t m = ballot((f >> j) & 1u);
      pre[j] = rank_in(m);
      if (lane == 0) wtot[w][j] = (int32_t)__builtin_popcountll(m);
    }
    __syncthreads();
    int64_t pos[NEST_MAXR + 1];
    for (int j = 0; j <= R; j++) {
      int64_t p = base[j] + pre[j];
      for (int v = 0; v < w; v++) p += wtot[v][j];
      pos[j] = p;
    }
    if (i < a.n) {
      const int d = a.def[i];
      for (int k = 1; k <= R; k++) {
        if ((f >> (k - 1)) & 1u) {  // a level-k list starts here
          const int64_t q = pos[k - 1];
          a.off[a.ostride * (k - 1) + q] = (int32_t)pos[k];
          if (d >= a.rdef[k] - 1) atomicOr(&a.val[a.vstride * (k - 1) + (q >> 5)], 1u << (q & 31));
        }
      }
      if ((f >> R) & 1u && d == a.max_def) {
        const int64_t q = pos[R];
        atomicOr(&a.val[a.vstride * R + (q >> 5)], 1u << (q & 31));
      }
    }
    __syncthreads();
    if ((int)threadIdx.x <= R) {
      int64_t t = 0;
      for (int v = 0; v < 4; v++) t += wtot[v][threadIdx.x];
      base[threadIdx.x] += t;
    }
    __syncthreads();
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    for (int k = 1; k <= R; k++) a.off[a.ostride * (k - 1) + base[k - 1]] = (int32_t)base[k];
    for (int j = 0; j <= R; j++) a.cnt[j] = base[j];
  }
}

}  // namespace
}  // namespace pq

extern "C" int pq_launch_fail_which, pq_launch_fail_err;  // pq_kernels.hip

extern "C" int pq_launch_nest(const pq::NestArgs *a, hipStream_t s) {
  if (a->nblocks <= 0) return 0;
  hipLaunchKernelGGL(pq::k_nest_count, dim3((unsigned)a->nblocks), dim3(256), 0, s, *a);
  hipLaunchKernelGGL(pq::k_nest_write, dim3((unsigned)a->nblocks), dim3(256), 0, s, *a);
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  pq_launch_fail_which = 41;
  pq_launch_fail_err = (int)e;
  return 17;
}
