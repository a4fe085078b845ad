// Waves resident per CU as a function of the kernel's VGPR allocation:
// each 64-thread workgroup clobbers v[N-1] (so next_free_vgpr = N), records its
// CU and start time, and spins ~20 us; waves starting in the first 5 us are
// the first residency round.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <map>

#define KERN(N)                                                                          \
  __global__ void __launch_bounds__(64) k_occ_##N(unsigned long long *ts, int *cu) {    \
    asm volatile("" ::: "v" #N);                                                         \
    unsigned long long t0 = wall_clock64();                                              \
    if (threadIdx.x == 0) { ts[blockIdx.x] = t0; cu[blockIdx.x] = __smid(); }            \
    while (wall_clock64() - t0 < 2000) __builtin_amdgcn_s_sleep(10);                     \
  }
KERN(63) KERN(95) KERN(103) KERN(111) KERN(119) KERN(120) KERN(124) KERN(127)
#define KERNS(N, S)                                                                      \
  __global__ void __launch_bounds__(64) k_occs_##N##_##S(unsigned long long *ts, int *cu) { \
    asm volatile("" ::: "v" #N, "s" #S);                                                 \
    unsigned long long t0 = wall_clock64();                                              \
    if (threadIdx.x == 0) { ts[blockIdx.x] = t0; cu[blockIdx.x] = __smid(); }            \
    while (wall_clock64() - t0 < 2000) __builtin_amdgcn_s_sleep(10);                     \
  }
KERNS(124, 99) KERNS(95, 99) KERNS(124, 79) KERNS(124, 89)

struct Big { unsigned long long *ts; int *cu; char pad[1400]; };
__global__ void __launch_bounds__(64) k_occ_lds(unsigned long long *ts, int *cu) {
  __shared__ double buf[984];  // 7872 B
  asm volatile("" ::: "v124");
  buf[threadIdx.x] = threadIdx.x;
  __builtin_amdgcn_wave_barrier();
  unsigned long long t0 = wall_clock64();
  if (threadIdx.x == 0) { ts[blockIdx.x] = t0 + (unsigned long long)buf[63 - threadIdx.x] * 0; cu[blockIdx.x] = __smid(); }
  while (wall_clock64() - t0 < 2000) __builtin_amdgcn_s_sleep(10);
}
__global__ void __launch_bounds__(64) k_occ_big(Big b) {
  asm volatile("" ::: "v124");
  unsigned long long t0 = wall_clock64();
  if (threadIdx.x == 0) { b.ts[blockIdx.x] = t0; b.cu[blockIdx.x] = __smid(); }
  while (wall_clock64() - t0 < 2000) __builtin_amdgcn_s_sleep(10);
}
static Big g_big;
static void run_big(unsigned long long *ts, int *cu) { g_big.ts = ts; g_big.cu = cu; hipLaunchKernelGGL(k_occ_big, dim3(256 * 32), dim3(64), 0, 0, g_big); }
static void run_lds(unsigned long long *ts, int *cu) { hipLaunchKernelGGL(k_occ_lds, dim3(256 * 32), dim3(64), 0, 0, ts, cu); }
typedef void (*KF)(unsigned long long *, int *);
int main() {
  const int n = 256 * 32;
  unsigned long long *ts;
  int *cu;
  hipMalloc(&ts, n * 8);
  hipMalloc(&cu, n * 4);
  struct { const char *name; KF f; int nv; } ks[] = {
      {"64", k_occ_63, 64}, {"96", k_occ_95, 96}, {"104", k_occ_103, 104}, {"112", k_occ_111, 112},
      {"120", k_occ_119, 120}, {"121", k_occ_120, 121}, {"125", k_occ_124, 125}, {"128", k_occ_127, 128},
      {"125+s100", k_occs_124_99, 125}, {"96+s100", k_occs_95_99, 96}, {"125+s80", k_occs_124_79, 125},
      {"125+s90", k_occs_124_89, 125}, {"125+lds7872", nullptr, 1}, {"125+kernarg1.4k", nullptr, 2}};
  for (auto &k : ks) {
    if (k.f) hipLaunchKernelGGL(k.f, dim3(n), dim3(64), 0, 0, ts, cu);
    else if (k.nv == 1) run_lds(ts, cu);
    else run_big(ts, cu);
    hipDeviceSynchronize();
    std::vector<unsigned long long> t(n);
    std::vector<int> c(n);
    hipMemcpy(t.data(), ts, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), cu, n * 4, hipMemcpyDeviceToHost);
    unsigned long long m = t[0];
    for (auto v : t) m = v < m ? v : m;
    std::map<int, int> per;
    for (int i = 0; i < n; i++)
      if (t[i] - m < 500) per[c[i]]++;
    int lo = 1 << 30, hi = 0;
    for (auto &p : per) { lo = p.second < lo ? p.second : lo; hi = p.second > hi ? p.second : hi; }
    printf("vgpr %s: first-round waves per CU min %d max %d over %zu CUs\n", k.name, lo, hi, per.size());
  }
  return 0;
}
