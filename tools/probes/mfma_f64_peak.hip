// Probe: sustained v_mfma_f64_16x16x4_f64 rate (back-to-back, 4 independent accumulators per
// wave, every CU busy) -> the fp64 matrix peak this box delivers.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(double* out, int iters) {
  d4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
  double x = threadIdx.x * 1e-3, y = 1.0 + blockIdx.x * 1e-6;
  for (int i = 0; i < iters; i++) {
    a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a2, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, a3, 0, 0, 0);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0[0] + a1[1] + a2[2] + a3[3];
}
int main() {
  int dev; hipGetDevice(&dev); hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
  const int blocks = p.multiProcessorCount * 4, threads = 64 * 2, iters = 20000;
  double* out; hipMalloc(&out, sizeof(double) * blocks * threads);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 100);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 16 * 16 * 4 * 4.0 * iters * (blocks * threads / 64);
  printf("CUs %d, fp64 MFMA 16x16x4: %.1f TFLOP/s (%.3f ms)\n", p.multiProcessorCount, flops / ms / 1e9, ms);
  return 0;
}
