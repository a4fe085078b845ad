// Latency of the move-direction math (cell.py:47-57) as k_tick_begin runs it:
// ~6k live cells, one lane each, so the kernel's time is one wave's dependent
// fp64 chain, and a wave with ONE lane on a slow path pays that path.
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I aigar_amd/csrc tools/micro/trig_latency.hip -o /tmp/trig_latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include <random>
#include <vector>

#include "aigar_trig.h"

using namespace aigar_math;

template <int M>
__global__ void __launch_bounds__(256) k(const double *x, const double *y, const double *m, double *o, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double xv = x[i], yv = y[i], mv = m[i];
  double r0 = 0, r1 = 0;
  if (M == 1) r0 = pow_glibc(mv, -0.35);
  if (M == 2) r0 = atan2_cr(yv, xv);
  if (M == 3) sincos_cr(xv * 0.006, r0, r1);
  if (M == 4 || M == 5) {
    const double a = atan2_cr(yv, xv);
    sincos_cr(a, r0, r1);
    if (M == 5) r0 *= pow_glibc(mv, -0.35);
  }
  if (M == 8) {
    const double a = atan2(yv, xv);
    sincos(a, &r0, &r1);
    r0 *= pow(mv, -0.35);
  }
  o[i] = r0 + r1;
}

template <int M>
float run(const double *x, const double *y, const double *m, double *o, int n, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 20; w++) hipLaunchKernelGGL(k<M>, dim3((n + 255) / 256), dim3(256), 0, 0, x, y, m, o, n);
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k<M>, dim3((n + 255) / 256), dim3(256), 0, 0, x, y, m, o, n);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.0f / reps;
}

// A, B alternating: with B's code in between, A starts from a cold instruction cache
template <int A, int B>
float run_pair(const double *x, const double *y, const double *m, double *o, int n, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < reps; r++) {
    hipLaunchKernelGGL(k<A>, dim3((n + 255) / 256), dim3(256), 0, 0, x, y, m, o, n);
    hipLaunchKernelGGL(k<B>, dim3((n + 255) / 256), dim3(256), 0, 0, x, y, m, o, n);
  }
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.0f / reps;
}

int main() {
  const int n = 6144, reps = 500;
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(-300.0, 300.0), um(10.0, 2000.0);
  std::vector<double> x(n), y(n), m(n);
  for (int i = 0; i < n; i++) {
    x[i] = u(g);
    y[i] = u(g);
    m[i] = um(g);
  }
  double *dx, *dy, *dm, *dout;
  hipMalloc(&dx, n * 8);
  hipMalloc(&dy, n * 8);
  hipMalloc(&dm, n * 8);
  hipMalloc(&dout, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(dy, y.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(dm, m.data(), n * 8, hipMemcpyHostToDevice);
  printf("us per launch (n=%d lanes, back-to-back launches)\n", n);
  printf("empty           %.2f\n", run<0>(dx, dy, dm, dout, n, reps));
  printf("pow             %.2f\n", run<1>(dx, dy, dm, dout, n, reps));
  printf("atan2_cr        %.2f\n", run<2>(dx, dy, dm, dout, n, reps));
  printf("sincos_cr       %.2f\n", run<3>(dx, dy, dm, dout, n, reps));
  printf("atan2+sincos    %.2f\n", run<4>(dx, dy, dm, dout, n, reps));
  printf("move direction  %.2f\n", run<5>(dx, dy, dm, dout, n, reps));
  printf("ocml            %.2f\n", run<8>(dx, dy, dm, dout, n, reps));
  const float p58 = run_pair<5, 8>(dx, dy, dm, dout, n, reps), p88 = run_pair<8, 8>(dx, dy, dm, dout, n, reps);
  const float p55 = run_pair<5, 5>(dx, dy, dm, dout, n, reps);
  printf("pairs: move+ocml %.2f, ocml+ocml %.2f, move+move %.2f -> move direction after other code %.2f vs warm %.2f\n",
         p58, p88, p55, p58 - p88 / 2, p55 / 2);
  return 0;
}
