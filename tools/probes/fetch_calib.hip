// FETCH_SIZE / WRITE_SIZE calibration probe (MI355X_MICROARCH.md §HBM: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").  Each kernel reads
// (or writes) every byte of a 1 GiB buffer exactly once — past the 256 MiB Infinity Cache — with
// one access pattern; rocprofv3 --pmc FETCH_SIZE (WRITE_SIZE) per dispatch / 2^30 is that
// pattern's counter-to-bytes ratio.  Patterns are the engine's:
//   rd16  16 B per lane, coalesced (the guide's calibrated case: expect 0.5)
//   rd8   8 B per lane, coalesced (feature rows read as doubles)
//   rd4   4 B per lane, coalesced (float32 embedding rows)
//   rd8t  8 B per lane in a 16-row x 4-column tile of doubles, rows 2048 doubles apart (the
//         A/B operand load of v_mfma_f64_16x16x4f64 in ss_nn_kernel / boost_embcost_kernel)
//   wr8   8 B per lane coalesced stores;  wr16  16 B per lane coalesced stores
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/fetch_calib tools/probes/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

static constexpr size_t BYTES = size_t(1) << 30;
static constexpr int BLOCK = 256;

// a data-dependent sink so the loads are not removed
__global__ void rd16(const double2* __restrict__ p, size_t n, double* sink) {
  double a = 0;
  for (size_t i = blockIdx.x * (size_t)BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK)
    a += p[i].x + p[i].y;
  if (a == 1.2345) sink[0] = a;
}
__global__ void rd8(const double* __restrict__ p, size_t n, double* sink) {
  double a = 0;
  for (size_t i = blockIdx.x * (size_t)BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK)
    a += p[i];
  if (a == 1.2345) sink[0] = a;
}
__global__ void rd4(const float* __restrict__ p, size_t n, double* sink) {
  float a = 0;
  for (size_t i = blockIdx.x * (size_t)BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK)
    a += p[i];
  if (a == 1.2345f) sink[0] = a;
}
// rows of F doubles; a wave owns a 16-row band and walks its columns 4 at a time: lane l reads
// row (l & 15), column k + (l >> 4) — one v_mfma_f64_16x16x4f64 operand per step
__global__ void rd8t(const double* __restrict__ p, int rows, int F, double* sink) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * BLOCK + threadIdx.x) >> 6;
  const int nwaves = gridDim.x * BLOCK / 64;
  double a = 0;
  for (int band = wave; band < rows / 16; band += nwaves) {
    const double* r = p + (size_t)(band * 16 + (lane & 15)) * F + (lane >> 4);
    for (int k = 0; k < F; k += 4) a += r[k];
  }
  if (a == 1.2345) sink[0] = a;
}
__global__ void wr8(double* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK)
    p[i] = (double)i;
}
__global__ void wr16(double2* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK)
    p[i] = make_double2((double)i, 1.0);
}

int main() {
  void* buf;
  double* sink;
  CK(hipMalloc(&buf, BYTES));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 0, BYTES));
  const int grid = 256 * 16;
  const int F = 2048, rows = (int)(BYTES / 8 / F);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; rep++) {  // rep 0 warms the code objects; rep 1 is the one to read
    float ms[6];
    int k = 0;
#define RUN(launch)                         \
  CK(hipEventRecord(e0));                   \
  launch;                                   \
  CK(hipEventRecord(e1));                   \
  CK(hipEventSynchronize(e1));              \
  CK(hipEventElapsedTime(&ms[k++], e0, e1));
    RUN(hipLaunchKernelGGL(rd16, dim3(grid), dim3(BLOCK), 0, 0, (const double2*)buf, BYTES / 16, sink));
    RUN(hipLaunchKernelGGL(rd8, dim3(grid), dim3(BLOCK), 0, 0, (const double*)buf, BYTES / 8, sink));
    RUN(hipLaunchKernelGGL(rd4, dim3(grid), dim3(BLOCK), 0, 0, (const float*)buf, BYTES / 4, sink));
    RUN(hipLaunchKernelGGL(rd8t, dim3(grid), dim3(BLOCK), 0, 0, (const double*)buf, rows, F, sink));
    RUN(hipLaunchKernelGGL(wr8, dim3(grid), dim3(BLOCK), 0, 0, (double*)buf, BYTES / 8));
    RUN(hipLaunchKernelGGL(wr16, dim3(grid), dim3(BLOCK), 0, 0, (double2*)buf, BYTES / 16));
    if (rep == 1) {
      const char* nm[6] = {"rd16", "rd8", "rd4", "rd8t", "wr8", "wr16"};
      for (int i = 0; i < 6; i++)
        printf("%-5s %8.3f ms  %7.1f GB/s  bytes %zu\n", nm[i], ms[i], BYTES / (ms[i] * 1e6), BYTES);
    }
  }
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
