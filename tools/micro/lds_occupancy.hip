// LDS-limited residency: 256-thread workgroups declaring S bytes of LDS, each
// spinning ~20 us; how many start in the first round on each CU?  (k_food_prep
// at 18.9 KB per block showed only 3 resident blocks per CU.)
// hipcc --offload-arch=gfx950 -O3 tools/micro/lds_occupancy.hip -o micro_bin/lds_occupancy
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
template <int S>
__global__ void __launch_bounds__(256) k(unsigned long long *ts, int *cu) {
  __shared__ char buf[S];
  buf[threadIdx.x * (S / 256)] = (char)threadIdx.x;
  __syncthreads();
  unsigned long long t0 = wall_clock64();
  if (threadIdx.x == 0) {
    ts[blockIdx.x] = t0 + (unsigned long long)buf[(threadIdx.x * 7) % S] * 0;
    cu[blockIdx.x] = __smid();
  }
  while (wall_clock64() - t0 < 2000) __builtin_amdgcn_s_sleep(10);
}
template <int S>
void run(unsigned long long *ts, int *cu, int n) {
  hipLaunchKernelGGL(k<S>, dim3(n), dim3(256), 0, 0, ts, cu);
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
  printf("LDS %6d B/block: first-round blocks per CU min %d max %d over %zu CUs\n", S, lo, hi, per.size());
}
int main() {
  const int n = 256 * 10;
  unsigned long long *ts;
  int *cu;
  (void)hipMalloc(&ts, n * 8);
  (void)hipMalloc(&cu, n * 4);
  run<1024>(ts, cu, n);
  run<8192>(ts, cu, n);
  run<12288>(ts, cu, n);
  run<16384>(ts, cu, n);
  run<18944>(ts, cu, n);
  run<21504>(ts, cu, n);
  run<24576>(ts, cu, n);
  run<32768>(ts, cu, n);
  run<40960>(ts, cu, n);
  run<65536>(ts, cu, n);
  return 0;
}
