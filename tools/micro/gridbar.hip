// a grid-wide barrier inside one launch against a kernel
// boundary inside a graph, at the tick's block counts.
//
// Each "phase" is: every thread stores one int that a thread of ANOTHER block
// loads in the next phase (a real cross-block hand-off, as between the tick's
// launches).  Two ways to run P phases:
//   chain   P dependent launches of a one-phase kernel, captured in a graph
//   fused   ONE launch running the P phases with P - 1 grid barriers
// Barrier: XCD-hierarchical sense reversal -- every block's thread 0 drains its
// stores, releases at agent scope and arrives on its group's counter (group =
// blockIdx % 8, the XCD the dispatcher puts the block on); the group's last
// arriver resets the counter and arrives on the top counter; the top's last
// arriver resets it and bumps the 8 group generation words; each block polls
// its group's word (sc1 loads + s_sleep), then acquires.  A bounded spin sets
// an error word instead of hanging (the grid must be co-resident: checked with
// the occupancy API before launching).
// Wall time per replay from HIP events over 300 replays after 20 warm-ups.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 gridbar.hip -o gridbar
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

struct Bar {
  unsigned cnt[8 * 32];  // group counters, one 128-B line each
  unsigned top[32];
  unsigned gen[8 * 32];  // group generation words, one line each
  unsigned err[32];
};

__device__ __forceinline__ unsigned ld_sc1(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void grid_bar(Bar *b, int nblocks) {
  __shared__ int s_dummy;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int g = blockIdx.x & 7;
    const int ng = (nblocks - g + 7) >> 3;           // blocks in group g
    const int ngroups = nblocks < 8 ? nblocks : 8;   // groups with a block
    const unsigned gen0 = ld_sc1(&b->gen[g * 32]);  // (read before arriving: it flips only after every arrival)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned t = __hip_atomic_fetch_add(&b->cnt[g * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((int)t == ng - 1) {
      __hip_atomic_store(&b->cnt[g * 32], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned u = __hip_atomic_fetch_add(&b->top[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int)u == ngroups - 1) {
        __hip_atomic_store(&b->top[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        for (int k = 0; k < ngroups; k++)
          __hip_atomic_store(&b->gen[k * 32], gen0 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    int spin = 0;
    while (ld_sc1(&b->gen[g * 32]) == gen0) {
      __builtin_amdgcn_s_sleep(1);
      if (++spin > (1 << 22)) {
        __hip_atomic_store(&b->err[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    s_dummy = 0;
  }
  __syncthreads();
}

// phase k: read the value block (b + 1) % n stored in phase k - 1, store our own
__device__ __forceinline__ void phase(int *buf, int k, int n) {
  const int tid = threadIdx.x;
  const int src = (blockIdx.x + 1) % n;
  int v = 0;
  if (k > 0) v = buf[((k - 1) & 1) * n * 256 + src * 256 + tid];
  buf[(k & 1) * n * 256 + blockIdx.x * 256 + tid] = v + k;
}

__global__ void __launch_bounds__(256) k_phase(int *buf, int k) { phase(buf, k, gridDim.x); }
__global__ void __launch_bounds__(256) k_fused(int *buf, int P, Bar *b) {
  for (int k = 0; k < P; k++) {
    if (k) grid_bar(b, gridDim.x);
    phase(buf, k, gridDim.x);
  }
}

template <class F>
double per_replay(hipStream_t s, F launch, int R = 300) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  launch();
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 20; w++) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t a, e;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&e));
  CK(hipEventRecord(a, s));
  for (int r = 0; r < R; r++) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e, s));
  CK(hipEventSynchronize(e));
  float ms;
  CK(hipEventElapsedTime(&ms, a, e));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return ms * 1e3 / R;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int *buf;
  Bar *bar;
  CK(hipMalloc(&buf, 2 * 4096 * 256 * sizeof(int)));
  CK(hipMemset(buf, 0, 2 * 4096 * 256 * sizeof(int)));
  CK(hipMalloc(&bar, sizeof(Bar)));
  CK(hipMemset(bar, 0, sizeof(Bar)));
  int per_cu = 0, cus = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  cus = prop.multiProcessorCount;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_fused, 256, 0));
  printf("CUs %d, co-resident k_fused blocks per CU %d\n", cus, per_cu);
  const int P = 10;
  printf("%8s %14s %14s %14s %14s\n", "blocks", "chain us/rep", "fused us/rep", "us/boundary", "us/barrier");
  for (int nb : {16, 64, 256, 512, 1040, 2048}) {
    if (nb > per_cu * cus) {
      printf("%8d  (not co-resident: skipped)\n", nb);
      continue;
    }
    const double one = per_replay(s, [&] { k_phase<<<nb, 256, 0, s>>>(buf, 0); });
    const double chain = per_replay(s, [&] {
      for (int k = 0; k < P; k++) k_phase<<<nb, 256, 0, s>>>(buf, k);
    });
    const double fused = per_replay(s, [&] { k_fused<<<nb, 256, 0, s>>>(buf, P, bar); });
    unsigned err = 0;
    CK(hipMemcpy(&err, &bar->err[0], 4, hipMemcpyDeviceToHost));
    if (err) {
      printf("%8d  barrier timed out (error word set)\n", nb);
      return 1;
    }
    printf("%8d %14.2f %14.2f %14.2f %14.2f\n", nb, chain, fused, (chain - one) / (P - 1), (fused - one) / (P - 1));
  }
  return 0;
}
