// What makes a short kernel of the tick last ~6 us in the trace when its waves
// finish in ~1 us?  Graphs of 10 dependent launches of one kernel kind, replayed
// 200 times; wall time per launch from HIP events.  Kinds:
//   triv     one store per block                         (the boundary alone)
//   ticket   + the last-block ticket (drain, agent release, atomic, acquire)
//   dirty    every thread writes W bytes (L2 left dirty for the boundary)
//   chain    every wave walks D dependent loads over a 12 MB table
//   code     every wave runs a long straight-line code body (cold I-cache)
//   vgpr     the triv body with ~190 VGPRs reserved (2 waves per SIMD)
// hipcc --offload-arch=gfx950 -O3 -std=c++17 kfloor.hip -o kfloor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__device__ bool last_block(int *ticket, int nblocks) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == nblocks - 1;
    if (t == nblocks - 1) {
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  return s_last;
}

__global__ void __launch_bounds__(256) k_triv(int *p) {
  if (threadIdx.x == 0) p[blockIdx.x * 64] = blockIdx.x;
}
__global__ void __launch_bounds__(256) k_ticket(int *p, int *tk) {
  if (threadIdx.x == 0) p[blockIdx.x * 64] = blockIdx.x;
  if (last_block(tk, gridDim.x) && threadIdx.x == 0) p[1] += 1;
}
__global__ void __launch_bounds__(256) k_dirty(double *p, int per_thread) {
  const size_t base = ((size_t)blockIdx.x * 256 + threadIdx.x);
  const size_t stride = (size_t)gridDim.x * 256;
  for (int k = 0; k < per_thread; k++) p[base + k * stride] = (double)k;
}
__global__ void __launch_bounds__(256) k_chain(const int *tab, int n, int depth, int *out, int passes = 1) {
  int i0 = (blockIdx.x * 256 + threadIdx.x) * 977 % n, i = i0, acc = 0;
  for (int p = 0; p < passes; p++) {  // a second pass re-walks the same addresses (cache-warm)
    i = i0 + acc;
    for (int k = 0; k < depth; k++) i = tab[i];
    acc += (i == -7);
  }
  if (i == -7) out[0] = i;
}
// a long straight-line body: distinct constants keep the unrolled FMAs from folding
__global__ void __launch_bounds__(256) k_code(double *p, int reps) {
  double x = p[threadIdx.x & 63] + blockIdx.x;
  for (int r = 0; r < reps; r++) {
#pragma unroll
    for (int k = 0; k < 6000; k++) x = fma(x, 1.0000001 + k * 1e-9, (double)k * 3e-7);
  }
  if (x == 12345.0) p[0] = x;
}
__global__ void __launch_bounds__(256) k_vgpr(int *p, int opaque) {
  double v[90];
#pragma unroll
  for (int k = 0; k < 90; k++) v[k] = p[k * 8 + (threadIdx.x & 7)] * 1.5;
  if (opaque == 12345) {
#pragma unroll
    for (int k = 0; k < 90; k++) p[k] = (int)v[k];
  }
  if (threadIdx.x == 0) p[4096 + blockIdx.x * 64] = blockIdx.x;
}

template <class F>
double per_launch(hipStream_t s, F launch, int n = 10, int R = 200) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < n; i++) launch();
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 10; w++) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  for (int r = 0; r < R; r++) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return ms * 1e3 / (R * n);
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int *p, *tk, *tab, *tabS;
  double *big;
  const int NT = 12 << 20 >> 2;  // 12 MB table of ints
  CK(hipMalloc(&p, 64 << 20));
  CK(hipMemset(p, 0, 64 << 20));
  CK(hipMalloc(&tk, 4096));
  CK(hipMemset(tk, 0, 4096));
  CK(hipMalloc(&big, 256 << 20));
  CK(hipMalloc(&tab, (size_t)NT * 4));
  {
    int *h = (int *)malloc((size_t)NT * 4);
    unsigned x = 12345;
    for (int i = 0; i < NT; i++) {
      x = x * 1664525u + 1013904223u;
      h[i] = (int)(x % NT);
    }
    CK(hipMemcpy(tab, h, (size_t)NT * 4, hipMemcpyHostToDevice));
    for (int i = 0; i < 16384; i++) h[i] %= 16384;  // a 64 KB table of its own
    CK(hipMalloc(&tabS, 16384 * 4));
    CK(hipMemcpy(tabS, h, 16384 * 4, hipMemcpyHostToDevice));
    free(h);
  }
  const int grids[] = {16, 256, 1024, 4096};
  for (int gi = 0; gi < 4; gi++) {
    const int G = grids[gi];
    printf("blocks %5d  triv %.2f  ticket %.2f  vgpr %.2f\n", G,
           per_launch(s, [&] { hipLaunchKernelGGL(k_triv, G, 256, 0, s, p); }),
           per_launch(s, [&] { hipLaunchKernelGGL(k_ticket, G, 256, 0, s, p, tk); }),
           per_launch(s, [&] { hipLaunchKernelGGL(k_vgpr, G, 256, 0, s, p, 0); }));
  }
  // dirty bytes left by each launch: G = 1024 blocks x 256 threads x 8 B x per
  for (int per : {1, 4, 16, 64}) {
    const double mb = 1024.0 * 256 * 8 * per / 1e6;
    printf("dirty %6.1f MB per launch: %.2f us\n", mb,
           per_launch(s, [&] { hipLaunchKernelGGL(k_dirty, 1024, 256, 0, s, big, per); }));
  }
  for (int depth : {1, 4, 8, 16}) {
    printf("chain depth %2d (1024 blocks): %.2f us   (16 blocks): %.2f us\n", depth,
           per_launch(s, [&] { hipLaunchKernelGGL(k_chain, 1024, 256, 0, s, tab, NT, depth, p); }),
           per_launch(s, [&] { hipLaunchKernelGGL(k_chain, 16, 256, 0, s, tab, NT, depth, p); }));
  }
  // is the L2 warm across a kernel boundary?  a 64 KB table (L2-resident) vs 12 MB,
  // one pass vs two passes over the same chain in one launch (the second pass is cache-warm)
  for (int nt : {16384, NT}) {
    for (int passes : {1, 2})
      printf("chain d16 table %8d B passes %d (256 blocks): %.2f us\n", nt * 4, passes,
             per_launch(s, [&] { hipLaunchKernelGGL(k_chain, 256, 256, 0, s, nt == NT ? tab : tabS, nt, 16, p, passes); }));
  }
  for (int reps : {0, 1}) {
    printf("code body reps %d (1024 blocks): %.2f us\n", reps,
           per_launch(s, [&] { hipLaunchKernelGGL(k_code, 1024, 256, 0, s, big, reps); }));
  }
  // the same chain kernel alone, back to back with itself vs interleaved with a dirtying kernel
  printf("chain d8 after dirty 8 MB (pairs, per pair): %.2f us\n",
         per_launch(s, [&] {
           hipLaunchKernelGGL(k_dirty, 1024, 256, 0, s, big, 4);
           hipLaunchKernelGGL(k_chain, 1024, 256, 0, s, tab, NT, 8, p);
         }));
  return 0;
}
