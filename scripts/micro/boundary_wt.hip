// Microbenchmark: cost of a dependent kernel boundary behind a kernel that leaves B bytes dirty in
// L2 (plain 16-B stores) vs writes them through (sc1 16-B stores), inside a hipGraph.
// Usage: ./boundary_wt   (prints us per (writer + tiny) pair for B = 0.5 .. 64 MB)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int WT>
__global__ __launch_bounds__(256) void writer(u32x4* __restrict__ out, long n16) {
  const u32x4 v = {1u, 2u, 3u, 4u};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256) {
    if (WT) {
      asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(out + i), "v"(v) : "memory");
    } else {
      out[i] = v;
    }
  }
}

__global__ void tiny(int* p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1; }

int main() {
  const long maxb = 64L << 20;
  u32x4* buf; int* flag;
  CK(hipMalloc(&buf, maxb));
  CK(hipMalloc(&flag, 64));
  hipStream_t s; CK(hipStreamCreate(&s));
  const int reps = 50, pairs = 20;
  for (int wt = 0; wt < 2; ++wt) {
    for (long mb2 : {1L, 4L, 16L, 32L, 64L, 128L}) {  // half-MB units
      const long bytes = mb2 << 19;
      const long n16 = bytes / 16;
      const int blocks = 2048;
      hipGraph_t g; hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int p = 0; p < pairs; ++p) {
        if (wt) hipLaunchKernelGGL(writer<1>, dim3(blocks), dim3(256), 0, s, buf, n16);
        else hipLaunchKernelGGL(writer<0>, dim3(blocks), dim3(256), 0, s, buf, n16);
        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, flag);
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
      hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
      CK(hipEventRecord(a, s));
      for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      printf("{\"stores\": \"%s\", \"MB\": %.1f, \"us_per_pair\": %.2f}\n", wt ? "sc1" : "plain", bytes / 1048576.0,
             ms * 1000.0 / reps / pairs);
      CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
