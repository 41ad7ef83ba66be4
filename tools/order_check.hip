// Does a kernel launched after another on the same non-blocking stream ever
// start before the first has finished?  A: one block, spins ~ms, writes flag.
// B: reads the flag.  Prints how many of N trials B saw the flag unset.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void kA(unsigned *flag, unsigned iters, unsigned *sink) {
  __shared__ unsigned lds[10000];
  unsigned x = threadIdx.x;
  for (unsigned i = 0; i < iters; i++) {
    lds[(x + i) % 10000] = x;
    x = x * 1664525u + 1013904223u + lds[(x * 7) % 10000];
  }
  if (threadIdx.x == 0 && x == 12345u) sink[0] = x;
  __syncthreads();
  if (threadIdx.x == 0) flag[0] = 1u;
}
__global__ void kB(const unsigned *flag, unsigned *out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = flag[0];
}
int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  unsigned *flag, *out, *sink;
  hipMalloc(&flag, 64); hipMalloc(&out, 64); hipMalloc(&sink, 64);
  int bad = 0;
  for (int t = 0; t < 200; t++) {
    hipMemsetAsync(flag, 0, 4, s);
    hipMemsetAsync(out, 0xff, 4, s);
    kA<<<1, 256, 0, s>>>(flag, 20000 + 100 * (t % 50), sink);
    kB<<<16, 64, 0, s>>>(flag, out);
    unsigned h = 0;
    hipMemcpyAsync(&h, out, 4, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    if (h != 1u) bad++;
  }
  printf("order_check: %d of 200 trials saw B run before A finished\n", bad);
  return 0;
}
