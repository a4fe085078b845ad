// How often do the device's atan2 / sin / cos (ocml) differ from the host's
// glibc results (what the reference's Python math calls)?  Inputs shaped like
// the stepper's: atan2 of command-point offsets, sin/cos of the resulting angles
// and of explosion angles (integer degrees).
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off trig_vs_glibc.hip -o trig_vs_glibc
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
__global__ void k(const double *y, const double *x, double *a, double *s, double *c, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  a[i] = atan2(y[i], x[i]);
  s[i] = sin(a[i]);
  c[i] = cos(a[i]);
}
int main() {
  const int n = 1 << 20;
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(-500.0, 500.0);
  std::vector<double> y(n), x(n), a(n), s(n), c(n);
  for (int i = 0; i < n; i++) { y[i] = u(g); x[i] = u(g); }
  double *dy, *dx, *da, *ds, *dc;
  hipMalloc(&dy, n * 8); hipMalloc(&dx, n * 8); hipMalloc(&da, n * 8); hipMalloc(&ds, n * 8); hipMalloc(&dc, n * 8);
  hipMemcpy(dy, y.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, dy, dx, da, ds, dc, n);
  hipMemcpy(a.data(), da, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(s.data(), ds, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(c.data(), dc, n * 8, hipMemcpyDeviceToHost);
  long ma = 0, msn = 0, mc = 0;
  for (int i = 0; i < n; i++) {
    double ha = std::atan2(y[i], x[i]);
    ma += ha != a[i];
    msn += std::sin(a[i]) != s[i];  // same argument on both sides
    mc += std::cos(a[i]) != c[i];
  }
  printf("n=%d atan2 mismatches %ld (%.4f%%), sin %ld (%.4f%%), cos %ld (%.4f%%)\n", n, ma, 100.0 * ma / n, msn,
         100.0 * msn / n, mc, 100.0 * mc / n);
  return 0;
}
