// Is a dependent load round in the tick slow because of address translation?
// The stepper allocates every field with its own hipMalloc (~100 arrays of a
// few hundred KB).  A kernel that loads one element from each of K such arrays
// (one round of independent loads) is timed in a graph of 10 launches that
// rotate over 4 disjoint sets of 32 arrays, with the arrays either separate
// hipMallocs or carved out of ONE allocation.  In-kernel: wall-clock per wave
// from entry to the round's completion (mean and max over waves).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tlb.hip -o tlb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

struct Ptrs {
  const double *p[32];
};
__global__ void __launch_bounds__(256) k_touch(Ptrs P, int K, int n, double *out, unsigned long long *ts) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  const int i = (int)(((long)gid * 7919) % n);
  const unsigned long long t0 = wall_clock64();
  double s = 0;
#pragma unroll
  for (int k = 0; k < 32; k++)
    if (k < K) s += P.p[k][i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t1 = wall_clock64();
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&ts[0], t1 - t0);
    atomicAdd(&ts[1], 1ull);
    atomicMax(&ts[2], t1 - t0);
  }
  if (s == -1.0) out[gid] = s;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int NA = 128;
  const size_t elems = 65536, bytes = elems * 8;  // 512 KB per array
  std::vector<double *> sep(NA);
  for (int k = 0; k < NA; k++) {
    CK(hipMalloc(&sep[k], bytes));
    CK(hipMemset(sep[k], 0, bytes));
  }
  double *big;
  CK(hipMalloc(&big, bytes * NA));
  CK(hipMemset(big, 0, bytes * NA));
  double *out;
  unsigned long long *ts;
  CK(hipMalloc(&out, 1 << 24));
  CK(hipMalloc(&ts, 64));
  for (int layout = 0; layout < 2; layout++)
    for (int grid : {16, 256})
      for (int K : {1, 8, 32}) {
        Ptrs sets[4];
        for (int q = 0; q < 4; q++)
          for (int k = 0; k < 32; k++) sets[q].p[k] = layout == 0 ? sep[q * 32 + k] : big + (size_t)(q * 32 + k) * elems;
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int l = 0; l < 12; l++) hipLaunchKernelGGL(k_touch, grid, 256, 0, s, sets[l % 4], K, (int)elems, out, ts);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int w = 0; w < 5; w++) CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipMemset(ts, 0, 64));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        const int R = 100;
        CK(hipEventRecord(a, s));
        for (int r = 0; r < R; r++) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        unsigned long long h[3];
        CK(hipMemcpy(h, ts, sizeof h, hipMemcpyDeviceToHost));
        printf("%s grid %3d K %2d: %.2f us/launch; wave round mean %.3f us max %.3f us\n",
               layout == 0 ? "separate" : "one-alloc", grid, K, ms * 1e3 / (R * 12), (double)h[0] / h[1] / 100.0,
               (double)h[2] / 100.0);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
      }
  return 0;
}
