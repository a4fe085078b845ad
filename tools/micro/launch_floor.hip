// Launch-floor microbenchmark: back-to-back dependent tiny kernels, graph vs stream,
// small vs ~1 KB kernel-argument blocks.  hipcc --offload-arch=gfx950 -O3 launch_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>
struct Big { int *p; long pad[122]; };
__global__ void k_small(int *p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1; }
__global__ void k_big(Big b) { if (threadIdx.x == 0 && blockIdx.x == 0) b.p[0] += 1; }
__global__ void k_ptr(const Big *b) { if (threadIdx.x == 0 && blockIdx.x == 0) b->p[0] += 1; }
__global__ void k_wide(int *p, int n) { int i = blockIdx.x * blockDim.x + threadIdx.x; if (i < n) p[i + 1] += 1; }
template <class F>
double run(hipStream_t s, F launch, int n, bool graph) {
  hipGraphExec_t ge = nullptr;
  if (graph) {
    hipGraph_t g;
    hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < n; i++) launch();
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphDestroy(g);
  }
  auto go = [&] { if (graph) hipGraphLaunch(ge, s); else for (int i = 0; i < n; i++) launch(); };
  for (int w = 0; w < 5; w++) go();
  hipStreamSynchronize(s);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a, s);
  const int R = 50;
  for (int r = 0; r < R; r++) go();
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  if (ge) hipGraphExecDestroy(ge);
  return ms * 1e3 / (R * n);
}
int main() {
  hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int *p; hipMalloc(&p, sizeof(int) * (1 << 22)); hipMemset(p, 0, 4 << 22);
  Big b{}; b.p = p; Big *db; hipMalloc(&db, sizeof(Big)); hipMemcpy(db, &b, sizeof b, hipMemcpyHostToDevice);
  const int n = 40;
  for (int graph = 0; graph < 2; graph++) {
    printf("%s small-arg 1 block : %.2f us/kernel\n", graph ? "graph " : "stream", run(s, [&] { hipLaunchKernelGGL(k_small, 1, 64, 0, s, p); }, n, graph));
    printf("%s 984B-arg 1 block  : %.2f us/kernel\n", graph ? "graph " : "stream", run(s, [&] { hipLaunchKernelGGL(k_big, 1, 64, 0, s, b); }, n, graph));
    printf("%s ptr-arg 1 block   : %.2f us/kernel\n", graph ? "graph " : "stream", run(s, [&] { hipLaunchKernelGGL(k_ptr, 1, 64, 0, s, (const Big *)db); }, n, graph));
    printf("%s 64K threads       : %.2f us/kernel\n", graph ? "graph " : "stream", run(s, [&] { hipLaunchKernelGGL(k_wide, 256, 256, 0, s, p, 65536); }, n, graph));
    printf("%s 1M threads        : %.2f us/kernel\n", graph ? "graph " : "stream", run(s, [&] { hipLaunchKernelGGL(k_wide, 4096, 256, 0, s, p, 1 << 20); }, n, graph));
  }
  return 0;
}
