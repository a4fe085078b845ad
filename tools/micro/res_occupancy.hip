// Residency of 256-thread workgroups by VGPR / SGPR / LDS use together
// (k_food_prep: 76 VGPR, 112 SGPR, 18.9 KB LDS showed ~3 resident blocks per CU).
// hipcc --offload-arch=gfx950 -O3 tools/micro/res_occupancy.hip -o micro_bin/res_occupancy
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
#define KERN(NAME, S, ...)                                                                   \
  __global__ void __launch_bounds__(256) NAME(unsigned long long *ts, int *cu) {             \
    __shared__ char buf[S];                                                                   \
    asm volatile("" ::: __VA_ARGS__);                                                                \
    buf[threadIdx.x * (S / 256)] = (char)threadIdx.x;                                         \
    __syncthreads();                                                                          \
    unsigned long long t0 = wall_clock64();                                                   \
    if (threadIdx.x == 0) {                                                                   \
      ts[blockIdx.x] = t0 + (unsigned long long)buf[(threadIdx.x * 7) % S] * 0;               \
      cu[blockIdx.x] = __smid();                                                              \
    }                                                                                         \
    while (wall_clock64() - t0 < 2000) __builtin_amdgcn_s_sleep(10);                          \
  }
KERN(k_v80, 256, "v79")
KERN(k_v80_l19, 18944, "v79")
KERN(k_v80_s100, 256, "v79", "s99")
KERN(k_v80_s100_l19, 18944, "v79", "s99")
KERN(k_v64_s100_l19, 18944, "v63", "s99")
KERN(k_v36_s100, 256, "v35", "s99")
typedef void (*KF)(unsigned long long *, int *);
void run(const char *name, KF f, unsigned long long *ts, int *cu, int n) {
  hipLaunchKernelGGL(f, dim3(n), dim3(256), 0, 0, ts, cu);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> t(n);
  std::vector<int> c(n);
  (void)hipMemcpy(t.data(), ts, n * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(c.data(), cu, n * 4, hipMemcpyDeviceToHost);
  unsigned long long m = t[0];
  for (auto v : t) m = v < m ? v : m;
  std::map<int, int> per;
  for (int i = 0; i < n; i++)
    if (t[i] - m < 500) per[c[i]]++;
  int lo = 1 << 30, hi = 0;
  for (auto &p : per) { lo = p.second < lo ? p.second : lo; hi = p.second > hi ? p.second : hi; }
  printf("%-18s first-round blocks per CU min %d max %d over %zu CUs\n", name, lo, hi, per.size());
}
int main() {
  const int n = 256 * 10;
  unsigned long long *ts;
  int *cu;
  (void)hipMalloc(&ts, n * 8);
  (void)hipMalloc(&cu, n * 4);
  run("v80", k_v80, ts, cu, n);
  run("v80 lds19k", k_v80_l19, ts, cu, n);
  run("v80 s100", k_v80_s100, ts, cu, n);
  run("v80 s100 lds19k", k_v80_s100_l19, ts, cu, n);
  run("v64 s100 lds19k", k_v64_s100_l19, ts, cu, n);
  run("v36 s100", k_v36_s100, ts, cu, n);
  return 0;
}
