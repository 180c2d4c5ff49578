// Probe: is v_mfma_f64_16x16x4_f64 a k-ordered fma chain (D = fma(a3,b3,fma(a2,b2,fma(a1,b1,fma(a0,b0,C)))))?
// Computes C = A (16xK) * B (Kx16) with K/4 chained MFMAs and compares with host fma chains.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k(const double* A, const double* B, double* C, int K) {
  const int lane = threadIdx.x;
  d4 acc = {0, 0, 0, 0};
  for (int s = 0; s < K; s += 4) {
    const double a = A[(lane & 15) * K + s + (lane >> 4)];
    const double b = B[(s + (lane >> 4)) * 16 + (lane & 15)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; r++) C[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = acc[r];
}

int main() {
  const int K = 2048;
  std::mt19937_64 g(7);
  std::normal_distribution<double> nd;
  double *A = (double*)malloc(8 * 16 * K), *B = (double*)malloc(8 * 16 * K), *C = (double*)malloc(8 * 256);
  for (int i = 0; i < 16 * K; i++) A[i] = nd(g), B[i] = nd(g);
  double *dA, *dB, *dC;
  hipMalloc(&dA, 8 * 16 * K); hipMalloc(&dB, 8 * 16 * K); hipMalloc(&dC, 8 * 256);
  hipMemcpy(dA, A, 8 * 16 * K, hipMemcpyHostToDevice);
  hipMemcpy(dB, B, 8 * 16 * K, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, K);
  hipMemcpy(C, dC, 8 * 256, hipMemcpyDeviceToHost);
  int eq_fma = 0, eq_fma_rev = 0, eq_muladd = 0, eq_pair = 0;
  double maxrel = 0;
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 16; j++) {
      double f = 0, fr = 0, m = 0, p = 0;
      for (int s = 0; s < K; s += 4) {
        for (int t = 0; t < 4; t++) f = std::fma(A[i * K + s + t], B[(s + t) * 16 + j], f);
        for (int t = 3; t >= 0; t--) fr = std::fma(A[i * K + s + t], B[(s + t) * 16 + j], fr);
        for (int t = 0; t < 4; t++) { volatile double pr = A[i * K + s + t] * B[(s + t) * 16 + j]; m = m + pr; }
        // pairwise: (p0+p1)+(p2+p3) exact-ish then added
        double q0 = A[i*K+s]*B[s*16+j], q1 = A[i*K+s+1]*B[(s+1)*16+j], q2 = A[i*K+s+2]*B[(s+2)*16+j], q3 = A[i*K+s+3]*B[(s+3)*16+j];
        p = p + ((q0 + q1) + (q2 + q3));
      }
      const double c = C[i * 16 + j];
      eq_fma += c == f; eq_fma_rev += c == fr; eq_muladd += c == m; eq_pair += c == p;
      maxrel = fmax(maxrel, fabs(c - f) / fabs(f));
    }
  printf("of 256: fma-chain k-order %d, fma-chain reversed %d, mul+add %d, pairwise-4 %d; max rel vs fma %.3g\n",
         eq_fma, eq_fma_rev, eq_muladd, eq_pair, maxrel);
  return 0;
}
