// probe: global_load_lds_dwordx4 LDS placement on gfx950 (M0 + lane*16 ?)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__shared__ __align__(16) double ring[2][1024];
__global__ void __launch_bounds__(64) k(const double* __restrict__ P, double* out) {
  const int lane = threadIdx.x;
  for (int i = lane; i < 2048; i += 64) (&ring[0][0])[i] = -1.0;
  __syncthreads();
  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) double*)&ring[0][0];
  for (int c = 0; c < 8; c++) {
    size_t a = (size_t)P + (size_t)c * 1024 + (size_t)lane * 16;
    const unsigned m = lds0 + c * 1024;
    unsigned sv;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(sv) : "v"(a), "s"(m) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = lane; i < 2048; i += 64) out[i] = (&ring[0][0])[i];
}
int main() {
  std::vector<double> h(2048);
  for (int i = 0; i < 2048; i++) h[i] = i;
  double *P, *o;
  hipMalloc(&P, 2048 * 8); hipMalloc(&o, 2048 * 8);
  hipMemcpy(P, h.data(), 2048 * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, P, o);
  std::vector<double> r(2048);
  hipMemcpy(r.data(), o, 2048 * 8, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 1024; i++) if (r[i] != i) { if (bad < 10) printf("slot[%d] = %g\n", i, r[i]); bad++; }
  printf("first 8: "); for (int i = 0; i < 8; i++) printf("%g ", r[i]); printf("\n");
  printf("bad %d of 1024; slot1[0..3] %g %g %g %g\n", bad, r[1024], r[1025], r[1026], r[1027]);
  return 0;
}
