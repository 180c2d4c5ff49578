// microbenchmark: one wave streaming R rows (8 KB each) of a matrix written by a previous
// kernel, with ~LQ=16 relax + wave-min work per row.  Variants:
//  0: 1-deep register prefetch   1: LDS DMA ring, m0 per chunk   2: DMA ring, m0 per 4 chunks
//  3: 2-deep register prefetch   4: no prefetch (load then use)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__shared__ __align__(16) double ring[4][1024];
__device__ __forceinline__ double wmin(double v) {
  for (int o = 32; o >= 1; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ void dma(size_t a, unsigned m) {
  unsigned sv;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(sv) : "v"(a), "s"(m) : "memory");
}
__device__ __forceinline__ void dma4(size_t a, unsigned m) {
  unsigned sv;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\t"
               "global_load_lds_dwordx4 %1, off offset:1024\n\t"
               "global_load_lds_dwordx4 %1, off offset:2048\n\t"
               "global_load_lds_dwordx4 %1, off offset:3072\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(sv) : "v"(a), "s"(m) : "memory");
}
template <int V>
__global__ void __launch_bounds__(64) k(const double* __restrict__ P, int R, int ld, double* out,
                                        unsigned long long* cyc) {
  const int lane = threadIdx.x;
  double vr[16], nx[16], nx2[16];
  for (int q = 0; q < 16; q++) vr[q] = 0.001 * (lane + 64 * q);
  double acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  auto rowp = [&](int r) { return (const char*)(P + (size_t)r * ld); };
  auto issue = [&](int r) {
    const size_t b = (size_t)rowp(r);
    const unsigned l0 = __builtin_amdgcn_readfirstlane(
        (unsigned)(size_t)(__attribute__((address_space(3))) double*)&ring[r & 3][0]);
    if (V == 1) {
      for (int c = 0; c < 8; c++) dma(b + c * 1024 + lane * 16, __builtin_amdgcn_readfirstlane(l0 + c * 1024));
    } else {
      dma4(b + lane * 16, l0);
      dma4(b + 4096 + lane * 16, __builtin_amdgcn_readfirstlane(l0 + 4096));
    }
  };
  if (V == 0 || V == 3) for (int q = 0; q < 16; q++) nx[q] = *(const double*)(rowp(0) + 8 * (lane + 64 * q));
  if (V == 3 && R > 1) for (int q = 0; q < 16; q++) nx2[q] = *(const double*)(rowp(1) + 8 * (lane + 64 * q));
  if (V == 1 || V == 2) for (int r = 0; r < 3 && r < R; r++) issue(r);
  for (int cur = 0; cur < R; cur++) {
    double rv[16];
    if (V == 1 || V == 2) {
      if (cur + 3 < R) issue(cur + 3);
      const int ahead = R - 1 - cur;
      if (ahead >= 3) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      else if (ahead == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int q = 0; q < 16; q++) rv[q] = ring[cur & 3][lane + 64 * q] - vr[q];
    } else if (V == 4) {
      for (int q = 0; q < 16; q++) rv[q] = *(const double*)(rowp(cur) + 8 * (lane + 64 * q)) - vr[q];
    } else {
      for (int q = 0; q < 16; q++) rv[q] = nx[q] - vr[q];
      if (V == 0 && cur + 1 < R) for (int q = 0; q < 16; q++) nx[q] = *(const double*)(rowp(cur + 1) + 8 * (lane + 64 * q));
      if (V == 3) {
        for (int q = 0; q < 16; q++) nx[q] = nx2[q];
        if (cur + 2 < R) for (int q = 0; q < 16; q++) nx2[q] = *(const double*)(rowp(cur + 2) + 8 * (lane + 64 * q));
      }
    }
    double m = rv[0];
    for (int q = 1; q < 16; q++) m = fmin(m, rv[q]);
    m = wmin(m);
    int cnt = 0;
    for (int q = 0; q < 16; q++) cnt += __popcll(__ballot(rv[q] == m));
    acc += m + cnt;
    vr[cur & 15] += 1e-9 * m;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = acc;
  if (lane == 0) cyc[0] = t1 - t0;
}
__global__ void fill(double* P, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) P[i] = (double)(i % 977) * 0.5;
}
int main() {
  const int R = 512, ld = 1024;
  const size_t n = (size_t)R * ld + 2048;
  double *P, *o, *junk;
  unsigned long long* cyc;
  hipMalloc(&P, n * 8); hipMalloc(&o, 64 * 8); hipMalloc(&cyc, 8);
  hipMalloc(&junk, (size_t)512 << 20);
  for (int v = 0; v < 5; v++) {
    for (int rep = 0; rep < 3; rep++) {
      hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, junk, ((size_t)512 << 20) / 8);  // evict MALL
      hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, P, n);
      switch (v) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, P, R, ld, o, cyc); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, P, R, ld, o, cyc); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, P, R, ld, o, cyc); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, P, R, ld, o, cyc); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(1), dim3(64), 0, 0, P, R, ld, o, cyc); break;
      }
      unsigned long long c = 0;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      printf("variant %d rep %d: %.0f cycles/row\n", v, rep, (double)c / R);
    }
  }
  return 0;
}
